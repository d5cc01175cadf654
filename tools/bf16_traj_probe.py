"""GPU diagnostic: the first steps of the reference loop (one synthetic
object, tests/test_gpu_converge.py's schedule) under HIP fp32, HIP bf16 and a
CPU emulation of the bf16 operand roundings (tools/bf16_rounding_emu.py's
Linear) from the SAME initial weights -- is the HIP bf16 trajectory what bf16
rounding alone predicts?

  python tools/bf16_traj_probe.py [steps] [init_seed]
"""
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def rb(t):
    return t.to(torch.bfloat16).to(torch.float32)


EMU = {"on": False}


class Lin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        xx, ww = (rb(x), rb(w)) if EMU["on"] else (x, w)
        ctx.save_for_backward(xx, ww)
        return xx @ ww.t() + b

    @staticmethod
    def backward(ctx, dy):
        xx, ww = ctx.saved_tensors
        d = rb(dy) if EMU["on"] else dy
        return (d @ ww, d.reshape(-1, d.shape[-1]).t() @ xx.reshape(-1, xx.shape[-1]),
                d.reshape(-1, d.shape[-1]).sum(0))


def main():
    from codenerf_amd.data import make_synthetic_srn
    from codenerf_amd.trainer import Trainer
    from test_gpu_converge import _hp
    from test_gpu_train import _oracle_training
    from oracle import ref_cpu
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    tmp = tempfile.mkdtemp()
    root = os.path.join(tmp, "data")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=1, n_views=1, H=32, W=32, focal=32.8, seed=11)
    runs, init = {}, None
    for prec in ("fp32", "bf16"):
        torch.manual_seed(seed)
        np.random.seed(seed)
        tr = Trainer("p" + prec, 0, hpams=_hp(root, prec), batch_size=256, check_iter=0, exp_root=tmp)
        if init is None:
            init = {"model": {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()},
                    "shape": tr.shape_codes.weight.detach().cpu().clone(),
                    "texture": tr.texture_codes.weight.detach().cpu().clone()}
        else:
            tr.model.load_state_dict(init["model"])
            with torch.no_grad():
                tr.shape_codes.weight.copy_(init["shape"])
                tr.texture_codes.weight.copy_(init["texture"])
        torch.manual_seed(1000 + seed)
        np.random.seed(1000 + seed)
        tr.training(0, steps, 1)
        runs[prec] = np.array(tr.psnr_log)
    torch.set_num_threads(16)
    orig = ref_cpu._lin

    def lin(p, name, x):
        if "latent" in name or name.startswith("sigma"):      # fp32 in the kernels
            return orig(p, name, x)
        return Lin.apply(x, p[name + ".weight"], p[name + ".bias"])
    ref_cpu._lin = lin
    for on in (False, True):
        EMU["on"] = on
        torch.manual_seed(1000 + seed)
        np.random.seed(1000 + seed)
        ps, _, _, _ = _oracle_training(_hp(root, "fp32"), init, steps, 256)
        runs["cpu_" + ("bf16emu" if on else "fp32")] = np.array(ps)
    for k, v in runs.items():
        print(f"{k:12s}", np.round(v, 3).tolist())
    ref = runs["cpu_fp32"]
    for k, v in runs.items():
        print(f"max |{k} - cpu_fp32| = {np.abs(v - ref).max():.4f}")


if __name__ == "__main__":
    main()
