"""CPU emulation: which operand split brings a bf16 training trajectory within
0.05 dB of the fp32 replay of the reference loop (src/trainer.py:34-96)?

Runs the oracle's replay (tests/test_gpu_train.py::_oracle_training) from the
same initial weights and RNG draws under ref_cpu.bf16_operands(...) variants:
  fp32 | bf16 (x, W, dy rounded) | W split (hi + lo) | W + x split | all split
Two regimes:
  one  -- tests/test_gpu_converge.py's object (1 object, 32^2, N=32): AdamW
          re-created every step (sign steps, chaotic);
  many -- N_OBJ objects, 64^2, N=64 over several epochs (Adam moments persist
          across the objects of an epoch; src/trainer.py:48-96).

  python tools/split_emu.py one|many [steps] [init seed; < 0: numpy-seeded params]
"""
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

B, S, F = "b", "s", "f"
VARIANTS = {
    "fp32": None,
    "bf16": dict(),
    "split_w": dict(split_w=True),
    "split_wx": dict(split_w=True, split_x=True),
    "split_all": dict(split_w=True, split_x=True, split_dy=True),
    # operand by operand: chain kernels (fw_*, bw_*) vs the dW pass (dw_*)
    "chain_s3": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S)),          # dW bf16
    "chain_f": dict(ops=dict(fw_w=F, fw_x=F, bw_w=F, bw_dy=F)),           # dW bf16
    "dw_f": dict(ops=dict(dw_x=F, dw_dy=F)),                               # chains bf16
    "fw_s": dict(ops=dict(fw_w=S, fw_x=S)),                                # forward only
    "w_dy": dict(ops=dict(fw_w=S, bw_w=S, bw_dy=S)),
    "bw_s3": dict(ops=dict(bw_w=S, bw_dy=S)),                              # dX chain only
    "bw_dy": dict(ops=dict(bw_dy=S)),
    "bw_w": dict(ops=dict(bw_w=S)),
    # the forward's W split only (x bf16), dX fully split
    "fwW_bw3": dict(ops=dict(fw_w=S, bw_w=S, bw_dy=S)),
}
# per-layer probes: chain_s3 everywhere except one layer in plain bf16
_LAYERS = ["encoding_xyz.0", "shape_layer_1.0", "shape_layer_2.0", "shape_layer_3.0", "encoding_shape",
           "encoding_viewdir.0", "texture_layer_1.0", "rgb.0", "rgb.2"]
for _l in _LAYERS:
    VARIANTS["s3_but_" + _l.split(".")[0]] = dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S),
                                                  layer_ops={_l: dict(fw_w=B, fw_x=B, bw_w=B, bw_dy=B)})
    VARIANTS["b16_but_" + _l.split(".")[0]] = dict(layer_ops={_l: dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S)})


def main():
    from codenerf_amd.data import make_synthetic_srn
    from oracle import ref_cpu
    from oracle.params import make_params, make_codes
    from test_gpu_train import _oracle_training
    regime = sys.argv[1] if len(sys.argv) > 1 else "one"
    torch.set_num_threads(os.cpu_count() or 8)
    tmp = tempfile.mkdtemp()
    root = os.path.join(tmp, "data")
    if regime == "one":
        from test_gpu_converge import _hp
        steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
        make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=1, n_views=1, H=32, W=32, focal=32.8, seed=11)
        hp, B, n_obj = _hp(root, "fp32"), 256, 1
    else:
        from test_gpu_regime import hp_many, N_OBJ, H, FOCAL
        steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3 * N_OBJ
        make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=N_OBJ, n_views=2, H=H, W=H, focal=FOCAL, seed=21)
        hp, B, n_obj = hp_many(root, "fp32"), 2048, N_OBJ
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if seed < 0:        # seeded numpy init (oracle.params)
        init = {"model": {k: torch.tensor(v) for k, v in make_params(-seed).items()}}
        s0, t0 = make_codes(-seed, n_obj)
        init["shape"], init["texture"] = torch.tensor(s0), torch.tensor(t0)
    else:               # the Trainer's own init sequence (make_model, make_codes) on the CPU
        from codenerf_amd.model import CodeNeRF
        torch.manual_seed(seed)
        np.random.seed(seed)
        m = CodeNeRF(**hp["net_hyperparams"])
        init = {"model": {k: v.detach().clone() for k, v in m.state_dict().items()},
                "shape": torch.randn(n_obj, 256) / np.sqrt(128), "texture": torch.randn(n_obj, 256) / np.sqrt(128)}
    runs = {}
    only = os.environ.get("EMU_ONLY")
    for name, cfg in VARIANTS.items():
        if only and name not in only.split(",") and name != "fp32":
            continue
        torch.manual_seed(1000 + max(seed, 0))
        np.random.seed(1000 + max(seed, 0))
        if cfg is None:
            ps, _, _, _ = _oracle_training(hp, init, steps, B)
        else:
            with ref_cpu.bf16_operands(**cfg):
                ps, _, _, _ = _oracle_training(hp, init, steps, B)
        runs[name] = np.array(ps)
        print(f"{name:10s}", np.round(runs[name], 3).tolist(), flush=True)
    ref = runs["fp32"]
    for k, v in runs.items():
        d = np.abs(v - ref)
        print(f"{k:10s} max |d| vs fp32 {d.max():.4f} dB; first step > 0.05: "
              f"{int(np.argmax(d > 0.05)) if (d > 0.05).any() else None}")


if __name__ == "__main__":
    main()
