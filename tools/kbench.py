"""Per-kernel timing of one C2 training step (128x128, 64 + 64 samples, bf16).

Fills the activation workspace with one real coarse + fine step, then times
each phase alone over `--reps` launches with HIP events on the launching
stream.  CODENERF_LIB selects a kernel variant build (make variant ...).
Also times a plain device copy (HBM calibration).

  python tools/kbench.py [--reps 20] [--only dw,fwd,bwd,copy]
"""
import argparse
import json
import math
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="fwd,bwd,dw,copy")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--dw-rows", default="", help="comma list of row counts: dW timed over rows [0, n) too")
    ap.add_argument("--weight-scale", type=float, default=1.0,
                    help="timing probe: scale every weight / code by this before timing (0: all-zero operands -- "
                         "the matrix cores' data-dependent power)")
    a = ap.parse_args()
    only = set(a.only.split(","))
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.trainer_core import TrainCore
    from bench import make_pose, FLOP_PER_SAMPLE, DW_FOLD_FLOP, DW_BYTES_PER_SAMPLE

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = CodeNeRF(3, 1, precision=a.precision).to(dev)
    sc = torch.nn.Parameter(torch.randn(4, 256, device=dev) / math.sqrt(128))
    tc = torch.nn.Parameter(torch.randn(4, 256, device=dev) / math.sqrt(128))
    core = TrainCore(model, sc, tc, near=0.8, far=1.8, n_coarse=64, n_fine=64)
    H = W = 128
    R = H * W
    gt = torch.rand(R, 3, device=dev)
    pose = make_pose(1.3, 30.0, 20.0).to(dev)
    # one step fills the workspace; a measurement variant may compute garbage
    # gradients, so the weights are restored before anything is timed
    saved = [p.detach().clone() for p in model.param_list() + [sc, tc]]
    core.train_step(H, W, 131.25, pose, gt, 0)
    torch.cuda.synchronize()
    with torch.no_grad():
        for p, q in zip(model.param_list() + [sc, tc], saved):
            p.copy_(q)
        if a.weight_scale != 1.0:
            for p in model.param_list() + [sc, tc]:
                p.mul_(a.weight_scale)
    step = core.step_impl
    eng = model.engine()
    params = model.param_list()
    eng.ensure_packed(params)
    Mc = R * 64
    M = eng.pad(Mc) + R * 64
    buf = step._ws[eng.device]
    cap = buf["cap"]
    blob, zvec = eng.latent_fwd(params, sc.detach()[0], tc.detach()[0])
    ro, vd = torch.rand(R, 3, device=dev), torch.nn.functional.normalize(torch.randn(R, 3, device=dev), dim=-1)
    ro = ro * 0.1 + torch.tensor([0.0, 0.4, 1.2], device=dev)
    z = torch.linspace(0.8, 1.8, 64, device=dev)
    out = {}
    if "fwd" in only:
        t = timeit(lambda: eng.mlp_fwd(blob, Mc, rays_o=ro, rays_d=vd, z=z, n_samples=64, act=buf["act"], act_M=cap,
                                       act_row0=0, sigma=buf["sig"][:eng.pad(Mc)], rgb=buf["rgb"][:eng.pad(Mc)]),
                   a.reps)
        out["fwd_ms"] = round(t, 4)
        out["fwd_tflops"] = round(FLOP_PER_SAMPLE["fwd"] * Mc / t / 1e9, 1)
        t = timeit(lambda: eng.mlp_fwd(blob, Mc, rays_o=ro, rays_d=vd, z=z, n_samples=64), a.reps)
        out["fwd_infer_ms"] = round(t, 4)
    if "bwd" in only:
        t = timeit(lambda: eng.mlp_bwd(blob, M, buf["dsig"], buf["drgb"], buf["act"], act_M=cap), a.reps)
        out["bwd_ms"] = round(t, 4)
        out["bwd_tflops"] = round(FLOP_PER_SAMPLE["bwd"] * M / t / 1e9, 1)
    if "dw" in only:
        grads = [torch.zeros_like(p) for p in params]
        t = timeit(lambda: eng.mlp_dw(buf["act"], M, zvec, grads, buf["dbuf"], buf["dw"], act_M=cap), a.reps)
        out["dw_ms"] = round(t, 4)
        out["dw_tflops"] = round((FLOP_PER_SAMPLE["dw"] * M + DW_FOLD_FLOP) / t / 1e9, 1)
        es = "fp32" if a.precision == "fp32" else "bf16"
        out["dw_alg_GBs"] = round(M * DW_BYTES_PER_SAMPLE[es] / t / 1e6, 1)    # operand bytes (srncar net, folded)
        for n in [int(x) for x in a.dw_rows.split(",") if x]:
            n = min(n, M)
            t = timeit(lambda: eng.mlp_dw(buf["act"], n, zvec, grads, buf["dbuf"], buf["dw"], act_M=cap), a.reps)
            out[f"dw_ms_{n}"] = round(t, 4)
    if "copy" in only:
        x = torch.empty(2 * 1024 ** 3, dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)
        t = timeit(lambda: y.copy_(x), 10)
        out["copy_GBs"] = round(2 * x.numel() / t / 1e6, 1)
        xf = x.view(torch.float32)
        t = timeit(lambda: xf.fill_(1.0), 10)
        out["fill_GBs"] = round(x.numel() / t / 1e6, 1)
        acc = torch.empty(1, device=dev)
        t = timeit(lambda: torch.sum(xf, dim=0, out=acc), 10)
        out["read_GBs"] = round(x.numel() / t / 1e6, 1)
    out["lib"] = os.environ.get("CODENERF_LIB", "default")
    out["precision"] = a.precision
    out["weight_scale"] = a.weight_scale
    print(json.dumps(out))


if __name__ == "__main__":
    main()
