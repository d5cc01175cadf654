"""Per-tensor trace: does the HIP bf16x3 step compute what its emulation
(oracle/ref_cpu.py ``bf16_operands(ops=OPS_BF16X3)``) computes?  (round-4
verdict item 1: seed 3 of tests/test_gpu_regime.py's many-object regime.)

At states along a HIP fp32 trajectory of that regime (8 objects, 64^2, 64
samples, srncar.json rates), one training image of the object the loop
visits at that step is run through

  x3     HIP bf16x3 (render.ImageStep, the trainer's own step)
  f32    HIP fp32
  emuG   the emulation of bf16x3 in torch on the GPU
  emuC   the same emulation on the CPU (a second fp32 summation order)
  t32    the fp32 reference (oracle) on the CPU
  f64    the reference in float64 (ground truth)

and, per parameter / code tensor, prints the rel-L2 of each against f64 and
the pairs that tell an arithmetic mismatch from rounding noise:

  x3~emuG   vs  emuG~emuC : the kernel against its emulation, beside the
                            emulation against itself under another order
  corr(x3 - f64, emuG - f64): ~1 when the kernel rounds the operands the
                            emulation rounds (the dominant error is the
                            deterministic bf16 rounding of dW's dA operand)

  python tools/x3_trace.py OUT.json SEED STEP [STEP ...]
"""
import json
import os
import sys
import tempfile
import pathlib

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def _rel(a, b):
    a = a.detach().double().cpu().reshape(-1)
    b = b.detach().double().cpu().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-300))


def _corr(a, b, ref):
    ea = (a.detach().double().cpu() - ref.detach().double().cpu()).reshape(-1)
    eb = (b.detach().double().cpu() - ref.detach().double().cpu()).reshape(-1)
    return float((ea * eb).sum() / (ea.norm() * eb.norm() + 1e-300))


def hip_step(prec, sd, shape, tex, oi, ro, vd, z, gt, chunk):
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.render import ImageStep
    dev = torch.device("cuda", 0)
    m = CodeNeRF(3, 1, precision=prec)
    m.load_state_dict(sd)
    m = m.to(dev)
    st = torch.nn.Parameter(shape.clone().to(dev))
    tt = torch.nn.Parameter(tex.clone().to(dev))
    step = ImageStep(m, chunk=chunk, reg_coef=1e-4)
    losses, _, _ = step.forward_backward(ro.to(dev), vd.to(dev), z.to(dev), gt.to(dev), st, tt, oi)
    torch.cuda.synchronize()
    g = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
    g["shape_code"] = st.grad[oi].detach().cpu().clone()
    g["texture_code"] = tt.grad[oi].detach().cpu().clone()
    return g, losses.cpu().numpy()


def oracle_step(sd, shape, tex, oi, ro, vd, z, gt, chunk, dtype=torch.float32, device="cpu", ops=None,
                layer_ops=None):
    from oracle import ref_cpu
    p = {k: v.to(device, dtype).clone().requires_grad_() for k, v in sd.items()}
    st = shape.to(device, dtype).clone().requires_grad_()
    tt = tex.to(device, dtype).clone().requires_grad_()
    f = lambda t: t.to(device, dtype)
    args = (p, st, tt, oi, f(ro), f(vd), f(z), f(gt))
    if ops is None:
        losses, _ = ref_cpu.image_step(*args, chunk=chunk)
    else:
        with ref_cpu.bf16_operands(ops=ops, layer_ops=layer_ops):
            losses, _ = ref_cpu.image_step(*args, chunk=chunk)
    g = {k: v.grad.detach().cpu().clone() for k, v in p.items()}
    g["shape_code"] = st.grad[oi].detach().cpu().clone()
    g["texture_code"] = tt.grad[oi].detach().cpu().clone()
    return g, np.array(losses)


def main():
    import test_gpu_regime as R
    from codenerf_amd.data import SRN, collate_one
    from oracle import ref_cpu
    out, seed, steps = sys.argv[1], int(sys.argv[2]), [int(s) for s in sys.argv[3:]]
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    tmp = pathlib.Path(tempfile.mkdtemp())
    root = R._data(tmp)
    hp = R.hp_many(root, "fp32")
    rows = []
    init = None
    for k in steps:
        if k == 0:
            _, init = R._run(tmp, root, "fp32", 0, init, seed=seed)
        else:
            _, init = R._run(tmp, root, "fp32", k, init, seed=seed)
        tr = R._run.last
        sd = {n: v.detach().cpu().clone() for n, v in tr.model.state_dict().items()}
        shape = tr.shape_codes.weight.detach().cpu().clone()
        tex = tr.texture_codes.weight.detach().cpu().clone()
        oi = k % R.N_OBJ
        ds = SRN("srn_cars", "cars_train", root, 1, crop_img=False, n_train_views=2)
        np.random.seed(5000 + k)
        focal, H, W, imgs, poses, _, _ = collate_one(ds[oi])
        ro, vd = ref_cpu.get_rays(int(H), int(W), focal, poses[0, 0])
        g = torch.Generator().manual_seed(7000 + k)
        z = ref_cpu.stratified_z(hp["near"], hp["far"], hp["N_samples"], jitter=torch.rand(hp["N_samples"],
                                                                                           generator=g))
        gt = imgs[0, 0].contiguous()
        args = (sd, shape, tex, oi, ro, vd, z, gt, R.B)
        res = {}
        res["x3"], lx3 = hip_step("bf16x3", *args)
        res["f32"], _ = hip_step("fp32", *args)
        emu = dict(ops=ref_cpu.OPS_BF16X3_K, layer_ops=ref_cpu.X3_LAYER_OPS)
        res["emuG"], _ = oracle_step(*args, device="cuda", **emu)
        res["emuC"], _ = oracle_step(*args, **emu)
        res["t32"], _ = oracle_step(*args)
        res["f64"], l64 = oracle_step(*args, dtype=torch.float64)
        f64 = res["f64"]
        print(f"\nseed {seed} step {k} object {oi}: chunk losses x3 {np.round(lx3, 6).tolist()} f64 "
              f"{np.round(l64, 6).tolist()}")
        hdr = (f"{'tensor':28s} {'x3~f64':>9s} {'emuG~f64':>9s} {'emuC~f64':>9s} {'x3~emuG':>9s} "
               f"{'emuG~emuC':>9s} {'corr':>6s} {'f32~f64':>9s} {'t32~f64':>9s}")
        print(hdr)
        trow = {"seed": seed, "step": k, "object": oi, "tensors": {}}
        for name in f64:
            r = {"x3_f64": _rel(res["x3"][name], f64[name]), "emuG_f64": _rel(res["emuG"][name], f64[name]),
                 "emuC_f64": _rel(res["emuC"][name], f64[name]), "x3_emuG": _rel(res["x3"][name], res["emuG"][name]),
                 "emuG_emuC": _rel(res["emuG"][name], res["emuC"][name]),
                 "corr": _corr(res["x3"][name], res["emuG"][name], f64[name]),
                 "f32_f64": _rel(res["f32"][name], f64[name]), "t32_f64": _rel(res["t32"][name], f64[name])}
            trow["tensors"][name] = r
            print(f"{name:28s} {r['x3_f64']:9.2e} {r['emuG_f64']:9.2e} {r['emuC_f64']:9.2e} {r['x3_emuG']:9.2e} "
                  f"{r['emuG_emuC']:9.2e} {r['corr']:6.3f} {r['f32_f64']:9.2e} {r['t32_f64']:9.2e}", flush=True)
        rows.append(trow)
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
