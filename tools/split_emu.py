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

Env: EMU_ONLY=a,b (variants; fp32 always runs), EMU_THREADS, EMU_DEVICE
(e.g. cuda: the replay's tensors on a GPU -- torch fp32 matmuls, the same
host random draws), EMU_GS_LOG2 (the fp16 variants' gradient scale).
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
GS = float(2 ** int(os.environ.get("EMU_GS_LOG2", "20")))
VARIANTS = {
    "fp32": None,
    # fp32 through the emulation's own matmul path (x @ W^T + b instead of
    # F.linear): a second fp32 summation order -- the chaos floor
    "f_path": dict(ops=dict(fw_w=F, fw_x=F, bw_w=F, bw_dy=F, dw_x=F, dw_dy=F)),
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
    # bf16x3 chains + a split dW operand (round-4 verdict item 1)
    "s3_dwdy": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_dy=S)),
    "s3_dwx": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S)),
    "s3_dwall": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S, dw_dy=S)),
    # the built bf16x3 exactly: encoding_viewdir's dir-PE columns stay hi only
    # in dW (dw.hip: its LO slab would not fit the ring) -- and with the dW
    # upstream gradients split too
    "x3_kernel": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S),
                      layer_ops={"encoding_viewdir.0": dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S,
                                                            dw_x_split_cols=256)}),
    # ... with the latent path's gradient from the bf16 dA sums as the kernels
    # form it (dw.hip bias sums -> dz = W^T db, dW += db (x) z)
    "x3_kdb": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S, inj_dy=B),
                   layer_ops={"encoding_viewdir.0": dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S,
                                                         dw_x_split_cols=256)}),
    # ... and from an exact (split) sum
    "x3_ksdb": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S, inj_dy=S),
                    layer_ops={"encoding_viewdir.0": dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S,
                                                          dw_x_split_cols=256)}),
    "x3_kernel_dwall": dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S, dw_dy=S),
                            layer_ops={"encoding_viewdir.0": dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S,
                                                                  dw_dy=S, dw_x_split_cols=256)}),
    # weights plain bf16 (no W lo stream, 2 MFMAs per block: W_hi x_hi + W_hi x_lo),
    # chain operands split, dW X split -- in both chains / forward / dX only
    "wb_s2": dict(ops=dict(fw_w=B, fw_x=S, bw_w=B, bw_dy=S, dw_x=S)),
    "wb_fwd": dict(ops=dict(fw_w=B, fw_x=S, bw_w=S, bw_dy=S, dw_x=S)),
    "wb_bwd": dict(ops=dict(fw_w=S, fw_x=S, bw_w=B, bw_dy=S, dw_x=S)),
    # fp16 operands ("h": one fp16, "hs": fp16 hi + lo) with the backward's
    # gradients scaled by GS (a power of two) before rounding
    "h_all": dict(ops=dict(fw_w="h", fw_x="h", bw_w="h", bw_dy="h", dw_x="h", dw_dy="h", grad_scale=GS)),
    "h3_dwb": dict(ops=dict(fw_w="hs", fw_x="hs", bw_w="hs", bw_dy="hs", grad_scale=GS)),
    "h3_dwh": dict(ops=dict(fw_w="hs", fw_x="hs", bw_w="hs", bw_dy="hs", dw_x="h", dw_dy="h", grad_scale=GS)),
    "h3_dwhs": dict(ops=dict(fw_w="hs", fw_x="hs", bw_w="hs", bw_dy="hs", dw_x="hs", dw_dy="hs", grad_scale=GS)),
    "h3_noscale": dict(ops=dict(fw_w="hs", fw_x="hs", bw_w="hs", bw_dy="hs", dw_x="h", dw_dy="h")),
}
# bf16x3 chains + the dW X split, except ONE layer whose chain operands stay
# plain bf16 (which layers can skip the three-MFMA cost?); and the split in
# one chain direction only
_X3DWX = dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S, dw_x=S)
VARIANTS["dwx_fwd_only"] = dict(ops=dict(fw_w=S, fw_x=S, dw_x=S))
VARIANTS["dwx_bwd_only"] = dict(ops=dict(bw_w=S, bw_dy=S, dw_x=S))
VARIANTS["dwx_bwd_dy"] = dict(ops=dict(fw_w=S, fw_x=S, bw_dy=S, dw_x=S))
# per-layer probes: chain_s3 everywhere except one layer in plain bf16
_LAYERS = ["encoding_xyz.0", "shape_layer_1.0", "shape_layer_2.0", "shape_layer_3.0", "encoding_shape",
           "encoding_viewdir.0", "texture_layer_1.0", "rgb.0", "rgb.2"]
for _l in _LAYERS:
    # bf16x3 chains + ONE layer's dW operand split (which layers need it?)
    VARIANTS["s3_dwx_" + _l.replace(".0", "").replace(".", "")] = dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S),
                                                  layer_ops={_l: dict(dw_x=S)})
    VARIANTS["s3_dwdy_" + _l.replace(".0", "").replace(".", "")] = dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S),
                                                   layer_ops={_l: dict(dw_dy=S)})
    VARIANTS["dwx_but_" + _l.replace(".0", "").replace(".", "")] = dict(
        ops=dict(_X3DWX), layer_ops={_l: dict(fw_w=B, fw_x=B, bw_w=B, bw_dy=B)})
    VARIANTS["s3_but_" + _l.split(".")[0]] = dict(ops=dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S),
                                                  layer_ops={_l: dict(fw_w=B, fw_x=B, bw_w=B, bw_dy=B)})
    VARIANTS["b16_but_" + _l.split(".")[0]] = dict(layer_ops={_l: dict(fw_w=S, fw_x=S, bw_w=S, bw_dy=S)})


def main():
    from codenerf_amd.data import make_synthetic_srn
    from oracle import ref_cpu
    # the kernels' arithmetic op for op (round 5): + the three-MFMA products
    # (lo lo dropped) and the encoding_shape fold (ref_cpu.OPS_BF16X3_K)
    VARIANTS["x3_k"] = dict(ops=ref_cpu.OPS_BF16X3_K, layer_ops=ref_cpu.X3_LAYER_OPS)
    from oracle.params import make_params, make_codes
    from test_gpu_train import _oracle_training
    regime = sys.argv[1] if len(sys.argv) > 1 else "one"
    torch.set_num_threads(int(os.environ.get("EMU_THREADS", os.cpu_count() or 8)))
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
    import threading
    import time

    def beat():             # progress for a runner that kills silent commands
        t0 = time.time()
        while True:
            time.sleep(60)
            print(f"[split_emu] {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    runs = {}
    only = os.environ.get("EMU_ONLY")
    for name, cfg in VARIANTS.items():
        if only and name not in only.split(",") and name != "fp32":
            continue
        torch.manual_seed(1000 + max(seed, 0))
        np.random.seed(1000 + max(seed, 0))
        dev = os.environ.get("EMU_DEVICE")
        if cfg is None:
            ps, _, _, _ = _oracle_training(hp, init, steps, B, device=dev)
        else:
            with ref_cpu.bf16_operands(**cfg):
                ps, _, _, _ = _oracle_training(hp, init, steps, B, device=dev)
        runs[name] = np.array(ps)
        print(f"{name:10s}", np.round(runs[name], 3).tolist(), flush=True)
    ref = runs["fp32"]
    for k, v in runs.items():
        d = np.abs(v - ref)
        print(f"{k:10s} max |d| vs fp32 {d.max():.4f} dB; first step > 0.05: "
              f"{int(np.argmax(d > 0.05)) if (d > 0.05).any() else None}")
    if regime != "one":
        # epoch means (test_gpu_regime.py's long-horizon measure)
        em = {k: v[: len(v) // n_obj * n_obj].reshape(-1, n_obj).mean(1) for k, v in runs.items()}
        for k, v in em.items():
            g = np.abs(v - em["fp32"])
            first = int(np.argmax(g > 0.05)) if (g > 0.05).any() else None
            print(f"{k:10s} epoch-mean |d| vs fp32 {np.round(g, 3).tolist()} first epoch > 0.05: {first}",
                  flush=True)


if __name__ == "__main__":
    main()
