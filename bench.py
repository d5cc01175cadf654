"""Benchmark: CodeNeRF training throughput on MI355X (ray-samples / second).

Workload (BASELINE.json configs[1]): srncar.json network (3 shape blocks,
1 texture block, W = 256), one 128x128 image per object per step, 64 coarse
+ 64 fine samples per ray (128 MLP evaluations per ray), bf16 MFMA with fp32
accumulation, synthetic SRN-cars-like data (targets ray-cast from an
ellipsoid object by the SRN-format generator's renderer, cameras on a
radius-1.3 sphere, focal 131.25, near/far 0.8/1.8; no dataset is available
offline; --config c3 uses the srnchair.json geometry: near/far 1.25/2.75,
radius 2.0).  ``train_psnr`` is the last timed step's -10 log10(mean chunk
MSE) (src/trainer.py:99), averaged over ranks.  One step = rays -> samples -> CodeNeRF forward -> compositing +
chunk-mean MSE (+ code regulariser) -> full backward (dX chain, dW, latent
layers, code rows) -> [RCCL all-reduce of the gradients when N > 1] -> AdamW
over the model and both code tables.  ``value`` = ray-samples of all ranks /
max-over-ranks wall time of the K timed steps.

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py)
"""
import argparse
import json
import math
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BF16_PEAK_TFLOPS = 2500.0       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3        # fp32 MFMA
HBM_PEAK_GBS = 8000.0
FLOP_PER_SAMPLE = {"fwd": 899_328, "bwd": 853_248, "dw": 899_328}
DW_BYTES_PER_SAMPLE = 8_000     # bf16 dA + X operand planes read by dw_kernel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--n-coarse", type=int, default=64)
    ap.add_argument("--n-fine", type=int, default=64)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--objects", type=int, default=64)
    # other BASELINE configs, measured for DESIGN.md (the driver runs c2):
    #   c4: optimize.py test-time code optimisation, 50 views x 128^2 x 64
    #       samples per step, fwd + dX only (no weight gradients), bf16
    #   c5: 256^2, 128 + 128 samples, fp32, the image in 8 ray parts
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true",
                    help="one dX launch then one dW launch (no coarse/fine two-stream overlap)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    # rehearsal of the N > 1 path on a one-GPU box: gloo, every rank on cuda:0
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--one-device", action="store_true")
    return ap.parse_args()


def make_pose(radius, az_deg, el_deg):
    az, el = math.radians(az_deg), math.radians(el_deg)
    eye = torch.tensor([radius * math.cos(el) * math.sin(az), radius * math.sin(el),
                        radius * math.cos(el) * math.cos(az)], dtype=torch.float64)
    fwd = -eye / eye.norm()
    up = torch.tensor([0.0, 1.0, 0.0], dtype=torch.float64)
    right = torch.linalg.cross(fwd, up)
    right = right / right.norm()
    tup = torch.linalg.cross(right, fwd)
    c2w = torch.eye(4, dtype=torch.float64)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, tup, -fwd, eye
    return c2w.float()


class Timers:
    """HIP events around the kernels of one phase, on the launching stream."""

    def __init__(self):
        self.ev = {}
        self.on = False

    def mark(self, name):
        if not self.on:
            return None
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        return s

    def done(self, name, s):
        if s is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.ev.setdefault(name, []).append((s, e))

    def summary(self):
        """phase -> (mean ms per launch, total ms over the timed steps)"""
        out = {}
        for k, v in self.ev.items():
            tot = sum(s.elapsed_time(e) for s, e in v)
            out[k] = (tot / len(v), tot)
        return out


def main():
    args = parse()
    if args.config == "c4":
        args.H, args.n_coarse, args.n_fine, args.precision = 128, 64, 0, "bf16"
    elif args.config == "c5":
        args.H, args.n_coarse, args.n_fine, args.precision = 256, 128, 128, "fp32"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)     # RCCL over xGMI
        else:
            dist.init_process_group("gloo")

    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.trainer_core import TrainCore
    from codenerf_amd.dp import broadcast_from, object_for

    torch.manual_seed(1234 + rank)
    model = CodeNeRF(3, 1, precision=args.precision).to(dev)
    n_obj = args.objects
    shape_codes = torch.nn.Parameter(torch.randn(n_obj, 256, device=dev) / math.sqrt(128))
    texture_codes = torch.nn.Parameter(torch.randn(n_obj, 256, device=dev) / math.sqrt(128))
    # identical initial weights and codes on every rank
    broadcast_from(list(model.parameters()) + [shape_codes, texture_codes], dist)

    H = W = args.H
    focal = 131.25 * H / 128
    R = H * W
    timers = Timers()
    # C3 = srnchair.json geometry (near/far 1.25/2.75, cameras at radius 2.0)
    near, far, radius = (1.25, 2.75, 2.0) if args.config == "c3" else (0.8, 1.8, 1.3)
    core = TrainCore(model, shape_codes, texture_codes, near=near, far=far, n_coarse=args.n_coarse,
                     n_fine=args.n_fine, chunk=2048, reg_coef=1e-4, lr=(1e-4, 1e-3), timers=timers,
                     dist=dist)
    core.step_impl.overlap_dw = not args.no_overlap
    # synthetic views: a ray-cast ellipsoid object per rank (the SRN-format
    # generator's renderer, data.make_synthetic_srn) from poses on the sphere
    import numpy as np
    from codenerf_amd.data import _object_spec, _render_object
    g = torch.Generator(device="cpu").manual_seed(99 + rank)
    spec = _object_spec(np.random.Generator(np.random.PCG64(99 + rank)))
    n_views = 8

    def view():
        c2w = make_pose(radius, float(torch.rand(1, generator=g)) * 360 - 180,
                        float(torch.rand(1, generator=g)) * 50 - 10)
        img = _render_object(spec, c2w.double().numpy(), H, W, focal)
        return c2w.to(dev), torch.tensor(img.reshape(R, 3), dtype=torch.float32, device=dev)

    poses, gts = map(list, zip(*[view() for _ in range(n_views)]))
    ray_parts = 8 if args.config == "c5" else 1
    views_per_step = 50 if args.config == "c4" else 1
    if args.config == "c4":
        # src/optimizer.py:66-98: codes only (weights fixed), every target view
        # accumulates into the code gradients, then one AdamW step on the codes
        from codenerf_amd.optim import FusedAdamW
        from codenerf_amd.render import ImageStep
        from codenerf_amd import engine as _eng
        img = ImageStep(model, chunk=2048, reg_coef=1e-4, timers=timers)
        sc1 = torch.nn.Parameter(shape_codes.detach()[:1].clone())
        tc1 = torch.nn.Parameter(texture_codes.detach()[:1].clone())
        copt = FusedAdamW([{"params": [sc1], "lr": 1e-2}, {"params": [tc1], "lr": 1e-2}])
        extra = [view() for _ in range(50 - n_views)]
        poses += [e[0] for e in extra]
        gts += [e[1] for e in extra]

    last = {}

    def step(i):
        if args.config == "c4":
            sc1.grad = torch.zeros_like(sc1)
            tc1.grad = torch.zeros_like(tc1)
            for v in range(views_per_step):
                ro, vd = _eng.get_rays_dev(H, W, focal, True, poses[v])
                loss, _, _ = img.forward_backward(ro, vd, core.stratified_z(dev), gts[v], sc1, tc1, 0,
                                                  weight_grads=False)
                last.setdefault("views", []).append(loss)
            copt.step()
            last["losses"] = torch.cat(last.pop("views"))
            return
        v = i % n_views
        obj = object_for(i, rank, world, n_obj)
        last["losses"] = core.train_step(H, W, focal, poses[v], gts[v], obj, ray_parts=ray_parts)[0]

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    timers.on = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples_per_step = R * (args.n_coarse + args.n_fine) * views_per_step
    value = samples_per_step * world * args.steps / dt
    ms = dt / args.steps * 1e3

    # train PSNR of the last timed step (src/trainer.py:99: -10 log10 of the
    # mean of the chunk MSEs; the fine pass's losses when n_fine > 0)
    ls = last["losses"]
    ls = ls[1] if isinstance(ls, tuple) else ls
    train_psnr = float(-10 * torch.log10(ls.float().mean()))
    if dist is not None:
        t = torch.tensor([train_psnr], device=dev, dtype=torch.float64)
        dist.all_reduce(t)
        train_psnr = float(t.item()) / world

    summ = timers.summary()
    kern = {k: v[0] for k, v in summ.items()}                     # ms per launch
    per_step = {k: v[1] / args.steps for k, v in summ.items()}    # ms per step (all launches)
    peak = BF16_PEAK_TFLOPS if args.precision == "bf16" else FP32_PEAK_TFLOPS
    roof = None
    if kern:
        flops = {k: FLOP_PER_SAMPLE[k] * samples_per_step for k in FLOP_PER_SAMPLE if k in kern}
        if args.config == "c4":
            flops.pop("dw", None)       # codes-only: the dw timer brackets the bias sums
        overlapped = args.n_fine > 0 and core.step_impl.overlap_dw
        if overlapped:
            # the dX chain of the coarse rows and dW of the fine rows run
            # concurrently on two streams, so the phase spans overlap and the
            # longest span is not the limiter: report the dW launches (the
            # HBM-bound operand stream that bounds this design),
            # each timed from the moment its rows are ready to its end
            dom = "dw"
        else:
            dom = max(flops, key=lambda k: per_step[k])
        # algorithmic FLOPs of the phase per step / its launch time per step
        achieved = flops[dom] / (per_step[dom] * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": {"fwd": "chain_kernel<fwd,train>", "bwd": "chain_kernel<bwd>",
                                            "dw": "dw_kernel"}[dom],
                "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": load_traffic(args.config, dom),
                "ms_per_launch": {k: round(v, 4) for k, v in kern.items()},
                "ms_per_step_by_phase": {k: round(v, 4) for k, v in per_step.items()}}
        if overlapped:
            roof["overlap"] = ("2 dX + 2 dW launches per step: dX(fine rows); dX(coarse rows) || dW(fine rows) "
                               "on a second stream; dW(coarse rows); phase spans overlap")
        if dom == "dw" and args.precision == "bf16":
            # the weight-gradient pass streams the stored bf16 operands (dA and X
            # planes, 8,000 B per sample at the srncar net): its practical limiter
            dw_bytes = DW_BYTES_PER_SAMPLE * samples_per_step
            gbs = dw_bytes / (per_step["dw"] * 1e-3) / 1e9
            roof["hbm_view"] = {"bytes_per_launch": dw_bytes, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
        step_flops = sum(v for k, v in FLOP_PER_SAMPLE.items() if args.config != "c4" or k != "dw") * samples_per_step
        roof["step"] = {"achieved": round(step_flops / (ms * 1e-3) / 1e12, 2), "unit": "TFLOP/s",
                        "frac": round(step_flops / (ms * 1e-3) / 1e12 / peak, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_threads)

    if rank == 0:
        metric = {"c2": "ray-samples/sec (train step), SRN-cars 128x128, 64 coarse + 64 fine samples",
                  "c4": "ray-samples/sec (optimize.py code optimisation step), 50 views x 128x128 x 64 samples",
                  "c3": "ray-samples/sec (train step), SRN-chairs geometry 128x128, 64 coarse + 64 fine samples",
                  "c5": "ray-samples/sec (train step), SRN-cars 256x256, 128 coarse + 128 fine samples, fp32"}
        out = {
            "metric": metric[args.config],
            "value": round(value, 1), "unit": "ray-samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": f"synthetic ({H}x{W} ray-cast ellipsoid object per rank, poses on a radius-{radius} sphere, "
                    f"random-init weights)",
            "train_psnr": round(train_psnr, 3),
            "config": {"workload": f"{'srnchair' if args.config == 'c3' else 'srncar'}.json net, {H}x{W} image/object/step, {args.n_coarse}+{args.n_fine} "
                                   f"samples/ray, " + ("50 views, codes-only fwd+dX+AdamW" if args.config == "c4"
                                                       else "train step incl. AdamW"),
                       "name": args.config, "objects_per_step": world,
                       "rays_per_step_per_gpu": R, "parallelism": f"dp{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def load_traffic(config, kernel):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary of the same config (profiles/pmc_traffic.json), or None."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(config, {}).get(kernel)
    except OSError:
        return None


def cpu_baseline(threads):
    """The CPU oracle (torch fp32 restatement of the reference, pinned to its
    golden vectors) on a bounded sample: a 2048-ray chunk x 128 samples,
    forward + compositing + MSE + backward, timed on this host's cores."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle import ref_cpu
    from oracle.params import make_params
    torch.set_num_threads(threads)
    p = ref_cpu.param_tensors(make_params(0))
    s = (torch.randn(1, 256) / 11.3).requires_grad_()
    t = (torch.randn(1, 256) / 11.3).requires_grad_()
    B, N = 2048, 128
    ro = torch.zeros(B, 3) + torch.tensor([0.0, 0.4, 1.2])
    vd = torch.nn.functional.normalize(torch.randn(B, 3) * 0.2 + torch.tensor([0., -0.3, -1.]), dim=-1)
    z = torch.linspace(0.8, 1.8, N)
    gt = torch.rand(B, 3)

    def one():
        xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
        sig, rgb = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, N, -1), s, t)
        col, _ = ref_cpu.volume_rendering(sig, rgb, z)
        ((col - gt) ** 2).mean().backward()

    one()
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 10.0 or reps < 2:
        one()
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(B * N * reps / dt, 1), "unit": "ray-samples/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x (2048 rays x 128 samples) fwd+composite+MSE+backward, torch CPU fp32 oracle"}


if __name__ == "__main__":
    main()
