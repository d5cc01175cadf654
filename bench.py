"""Benchmark: CodeNeRF training throughput on MI355X (ray-samples / second).

Workload (BASELINE.json configs[1]): srncar.json network (3 shape blocks,
1 texture block, W = 256), one 128x128 image per object per step, 64 coarse
+ 64 fine samples per ray (128 MLP evaluations per ray), bf16 MFMA with fp32
accumulation -- by default the bf16x3f plan: the forward chains carry every
weight and activation as a bf16 hi + lo pair (three bf16 MFMAs per block:
rendered rgb within 1e-4 of the fp32 reference, the north-star bar), the
backward runs on bf16 operands; bf16, bf16x3 and fp32 are measured in the same
line (``precisions``) -- synthetic SRN-cars-like data (targets ray-cast from an
ellipsoid object by the SRN-format generator's renderer, cameras on a
radius-1.3 sphere, focal 131.25, near/far 0.8/1.8; no dataset is available
offline; --config c3 uses the srnchair.json geometry: near/far 1.25/2.75,
radius 2.0).  Train-PSNR parity (the metric's second half) is measured by
tests/test_gpu_converge.py and tests/test_gpu_regime.py, not here: a
random-init step's PSNR says nothing.  One step = rays -> samples -> CodeNeRF forward -> compositing +
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
# Algorithmic FLOPs per ray-sample of each pass: the
# forward and the dX chain as the reference's Linear layers; dW as this
# design computes it -- the reference's 13 weight GEMMs minus encoding_shape's
# 131,072, which dw_fold_kernel recovers per launch from the 257^2 fold
# operand (two 257 x 257 x 257 products, DW_FOLD_FLOP per launch).
FLOP_PER_SAMPLE = {"fwd": 899_328, "bwd": 853_248, "dw": 768_256}
DW_FOLD_FLOP = 2 * 2 * 257 ** 3
# Bytes per ray-sample the dW pass must read: the bf16 dA + X operand planes
# the forward / dX chains stored (encoding_shape folded).
DW_BYTES_PER_SAMPLE = {"bf16": 6_976, "bf16x3": 10_432, "bf16x3f": 6_976,
                       "fp32": 13_952}   # + the X lo planes in bf16x3; bf16x3f's dW is the bf16 one
PRECISIONS = ("bf16", "bf16x3", "bf16x3f", "fp32")
PRECISION_NOTE = {
    "bf16": "bf16 operands everywhere (rendered rgb ~2e-4 from the fp32 reference)",
    "bf16x3": "forward and dX chains on bf16 hi + lo operands and weights (3 MFMAs per block), dW on hi + lo X "
              "operands: fp32-class rgb and gradients",
    "bf16x3f": "the bf16x3 forward chains (fp32-class rendered rgb) + the bf16 backward (dX chain and dW on bf16 "
               "operands)",
    "fp32": "exact fp32 MFMA (v_mfma_f32_32x32x2_f32)",
}


def dtype_of(precision):
    """the arithmetic type the path computes in: MFMA operand type"""
    return "fp32" if precision == "fp32" else "bf16"
KERNEL_NAMES = {"fwd": "chain_kernel<fwd,train>", "bwd": "chain_kernel<bwd>", "dw": "dw_kernel"}
# algorithmic HBM bytes per ray of the fused ray-major step
# (24 B origin + direction in, 12 B gt, 12 B rgb out)
ALG_BYTES_PER_RAY = 48


def log(msg):
    """progress on stderr (a GPU runner kills a command that stays silent)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--n-coarse", type=int, default=64)
    ap.add_argument("--n-fine", type=int, default=64)
    ap.add_argument("--precision", default="bf16x3f", choices=list(PRECISIONS),
                    help="chain arithmetic: bf16 operands | bf16x3 (hi + lo operands, 3 MFMAs per block) | "
                         "bf16x3f (the bf16x3 forward, the bf16 backward) | fp32")
    ap.add_argument("--objects", type=int, default=64)
    ap.add_argument("--weights", default="weights/c2_regime_400.pth",
                    help="reference-format checkpoint (models.pth: model_params, shape/texture_code_params) to "
                         "start from (default: 400 steps of the srncar regime, tools/make_bench_weights.py -- the "
                         "step measured 1.3%% slower on them than on random-init weights, profiles/r04b_clock.md); "
                         "'none' = random init")
    # other BASELINE configs, measured for DESIGN.md (the driver runs c2):
    #   c4: optimize.py test-time code optimisation, 50 views x 128^2 x 64
    #       samples per step, fwd + dX only (no weight gradients), bf16
    #   c5: 256^2, 128 + 128 samples, fp32, the image in 8 ray parts
    #   c4eval: optimize.py's evaluation loop (src/optimizer.py:108-130): one
    #       step = one 128^2 view x 64 samples rendered forward-only + MSE
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c4eval", "c5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true",
                    help="one dX launch then one dW launch (no two-stream dX / dW pipelining)")
    ap.add_argument("--bwd-ranges", type=int, default=None, help="row ranges of the dX / dW pipeline")
    ap.add_argument("--dw-side-wgs", type=int, default=None,
                    help="persistent workgroups of the dW launches that run beside a dX chain (0: 256)")
    ap.add_argument("--no-fp32", action="store_true", help="skip the secondary precisions' figures of the C2 step")
    ap.add_argument("--recompute", action="store_true",
                    help="store-vs-recompute A/B: loss forwards store masks only, a second forward writes the dW planes")
    ap.add_argument("--cpu-baseline-only", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: OMP_NUM_THREADS, else all host CPUs)")
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
    """Per-kernel timers of the hot launches (chains, dW): two hipEvents per
    launch, recorded by the launch's own dispatch packet (cn_time_next_launch
    -> hipExtLaunchKernel) without a system-scope fence, so nothing sits
    between kernels (torch events around every launch added ~7 us each to the
    step)."""

    def __init__(self):
        self.ev = {}
        self.on = False
        self._hip = None

    def _rt(self):
        if self._hip is None:
            import ctypes
            h = ctypes.CDLL("libamdhip64.so.7")      # the process's HIP runtime (torch's, same SONAME)
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            self._hip = h
        return self._hip

    def _event(self):
        import ctypes
        e = ctypes.c_void_p()
        # hipEventDisableSystemFence: a timing event needs its timestamp, not
        # the system-scope release (an L2 write-back) a default event adds
        if self._rt().hipEventCreateWithFlags(ctypes.byref(e), 0x20000000) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")
        return e

    def record(self, e):
        """record e on the current stream"""
        import ctypes
        if self._rt().hipEventRecord(e, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def _ms(self, a, b):
        import ctypes
        ms = ctypes.c_float()
        if self._rt().hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def mark(self, name):
        """Arm the timer of the next hot launch (the caller launches it next)."""
        if not self.on:
            return None
        from codenerf_amd import _lib
        s, e = self._event(), self._event()
        if _lib.lib().cn_time_next_launch(s, e) != 0:
            raise RuntimeError("cn_time_next_launch failed")
        return (s, e)

    def done(self, name, s, n=0, contended=False):
        """n: samples the launch processed; contended: it shared the chip
        with a launch on another stream (render.ImageStep's dX / dW overlap)."""
        if s is None:
            return
        self.ev.setdefault(name, []).append((s[0], s[1], int(n), bool(contended)))

    def summary(self):
        """phase -> (mean ms per launch, total ms over the timed steps)"""
        out = {}
        for k, v in self.ev.items():
            tot = sum(self._ms(x[0], x[1]) for x in v)
            out[k] = (tot / len(v), tot)
        return out

    def split(self, name, contended):
        """(total ms, total samples, launches) over the phase's launches that
        did / did not share the chip"""
        v = [x for x in self.ev.get(name, []) if x[3] == contended]
        return sum(self._ms(x[0], x[1]) for x in v), sum(x[2] for x in v), len(v)


def build_workload(args, dev, rank, world, precision, timers, dist):
    """Model, codes, synthetic views and the step closure of one bench config."""
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.trainer_core import TrainCore
    from codenerf_amd.dp import broadcast_from, object_for

    torch.manual_seed(1234 + rank)
    model = CodeNeRF(3, 1, precision=precision).to(dev)
    n_obj = args.objects
    shape_codes = torch.nn.Parameter(torch.randn(n_obj, 256, device=dev) / math.sqrt(128))
    texture_codes = torch.nn.Parameter(torch.randn(n_obj, 256, device=dev) / math.sqrt(128))
    wpath = weights_path(args)
    if wpath:
        # trained weights (the reference's checkpoint keys, src/trainer.py:166-170);
        # the code tables repeat the checkpoint's objects
        ck = torch.load(wpath, map_location=dev, weights_only=True)
        model.load_state_dict(ck["model_params"])
        with torch.no_grad():
            for tab, key in ((shape_codes, "shape_code_params"), (texture_codes, "texture_code_params")):
                w = ck[key]["weight"].to(dev)
                tab.copy_(w[torch.arange(n_obj, device=dev) % w.shape[0]])
    # identical initial weights and codes on every rank
    broadcast_from(list(model.parameters()) + [shape_codes, texture_codes], dist)

    H = W = args.H
    focal = 131.25 * H / 128
    R = H * W
    # C3 = srnchair.json geometry (near/far 1.25/2.75, cameras at radius 2.0)
    near, far, radius = (1.25, 2.75, 2.0) if args.config == "c3" else (0.8, 1.8, 1.3)
    opts = dict(overlap_dw=not args.no_overlap)
    if args.bwd_ranges is not None:
        opts["bwd_ranges"] = args.bwd_ranges
    if args.dw_side_wgs is not None:
        opts["dw_side_wgs"] = args.dw_side_wgs
    core = TrainCore(model, shape_codes, texture_codes, near=near, far=far, n_coarse=args.n_coarse,
                     n_fine=args.n_fine, chunk=2048, reg_coef=1e-4, lr=(1e-4, 1e-3), timers=timers,
                     dist=dist, step_opts=opts)
    core.step_impl.recompute = bool(getattr(args, "recompute", False))
    # synthetic views: a ray-cast ellipsoid object per rank (the SRN-format
    # generator's renderer, data.make_synthetic_srn) from poses on the sphere
    import numpy as np
    from codenerf_amd.data import _object_spec, _render_object
    g = torch.Generator(device="cpu").manual_seed(99 + rank)
    spec = _object_spec(np.random.Generator(np.random.PCG64(99 + rank)))
    n_views = 50 if args.config in ("c4", "c4eval") else 8

    def view():
        c2w = make_pose(radius, float(torch.rand(1, generator=g)) * 360 - 180,
                        float(torch.rand(1, generator=g)) * 50 - 10)
        img = _render_object(spec, c2w.double().numpy(), H, W, focal)
        return c2w.to(dev), torch.tensor(img.reshape(R, 3), dtype=torch.float32, device=dev)

    poses, gts = map(list, zip(*[view() for _ in range(n_views)]))
    last = {}
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

        def step(i):
            sc1.grad = torch.zeros_like(sc1)
            tc1.grad = torch.zeros_like(tc1)
            views = []
            for v in range(n_views):
                ro, vd = _eng.get_rays_dev(H, W, focal, True, poses[v])
                loss, _, _ = img.forward_backward(ro, vd, core.stratified_z(dev), gts[v], sc1, tc1, 0,
                                                  weight_grads=False)
                views.append(loss)
            copt.step()
            last["losses"] = torch.cat(views)
    elif args.config == "c4eval":
        # src/optimizer.py:108-130: no_grad forward of a held-out view with
        # the optimised codes, composite, MSE (PSNR); the view rays come from
        # the pose on the device (get_rays), z from the host draw
        from codenerf_amd import engine as _eng
        eng = model.engine()
        params = model.param_list()
        eng.ensure_packed(params, bwd=False)
        blob, _ = eng.latent_fwd(params, shape_codes.detach()[0], texture_codes.detach()[0])
        M = R * args.n_coarse
        sig = torch.empty(eng.pad(M), device=dev)
        rgbs = torch.empty(eng.pad(M), 3, device=dev)

        def step(i):
            v = i % n_views
            ro, vd = _eng.get_rays_dev(H, W, focal, True, poses[v])
            z = core.stratified_z(dev)
            ev = timers.mark("fwd")
            eng.mlp_fwd(blob, M, rays_o=ro, rays_d=vd, z=z, n_samples=args.n_coarse, sigma=sig, rgb=rgbs)
            timers.done("fwd", ev, n=M)
            rgb, _ = _eng.composite_fwd(sig, rgbs, z, R, args.n_coarse)
            last["losses"] = ((rgb - gts[v]) ** 2).mean().reshape(1)
    else:
        def step(i):
            v = i % n_views
            obj = object_for(i, rank, world, n_obj)
            last["losses"] = core.train_step(H, W, focal, poses[v], gts[v], obj)[0]
    views_per_step = n_views if args.config == "c4" else 1
    samples_per_step = R * (args.n_coarse + args.n_fine) * views_per_step
    return dict(step=step, last=last, core=core, R=R, H=H, radius=radius, samples_per_step=samples_per_step)


def weights_path(args):
    """The checkpoint the bench starts from, or None (random init)."""
    if args.weights is None or args.weights.lower() == "none":
        return None
    p = args.weights if os.path.isabs(args.weights) else os.path.join(REPO, args.weights)
    if not os.path.exists(p):
        raise FileNotFoundError(p)
    return p


def timed_run(wl, steps, warmup, timers, dist, dev):
    """warmup untimed steps, then exactly `steps` steps between barriers +
    synchronize; per-step HIP events (current stream) give the median."""
    for i in range(warmup):
        wl["step"](i)
    torch.cuda.synchronize()
    log(f"warmup done ({warmup} steps); timing {steps} steps")
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    timers.on = True
    # per-step marks: fence-less events (Timers.record), not torch events,
    # whose system-scope release would add an L2 write-back to every step
    marks = [timers._event() for _ in range(steps + 1)]
    t0 = time.perf_counter()
    timers.record(marks[0])
    for i in range(steps):
        wl["step"](warmup + i)
        timers.record(marks[i + 1])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timers.on = False
    per = sorted(timers._ms(marks[i], marks[i + 1]) for i in range(steps))
    median = per[len(per) // 2] if steps % 2 else 0.5 * (per[steps // 2 - 1] + per[steps // 2])
    if dist is not None:
        t = torch.tensor([dt, median], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, median = float(t[0]), float(t[1])
    return dt, median


def main():
    args = parse()
    if args.config in ("c4", "c4eval"):
        args.H, args.n_coarse, args.n_fine = 128, 64, 0
    elif args.config == "c5":
        args.H, args.n_coarse, args.n_fine, args.precision = 256, 128, 128, "fp32"
    if args.cpu_baseline_only is not None:
        # child of cpu_baseline: the CPU oracle only, no device
        print(json.dumps(_cpu_baseline_at(args.cpu_baseline_only, args, args.cpu_seconds)))
        return
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

    timers = Timers()
    log(f"config {args.config}, precision {args.precision}, world {world}")
    wl = build_workload(args, dev, rank, world, args.precision, timers, dist)
    clock = {"before_warmup": clock_probe(dev)}
    dt, median = timed_run(wl, args.steps, args.warmup, timers, dist, dev)
    clock["after_timed"] = clock_probe(dev)
    samples_per_step = wl["samples_per_step"]
    value = samples_per_step * world * args.steps / dt
    ms = dt / args.steps * 1e3

    roof = roofline(args, timers, samples_per_step, ms, wl["core"].step_impl.overlap_dw)
    H, R, radius = wl["H"], wl["R"], wl["radius"]

    # the other precisions on the same C2 geometry (secondary figures): fp32
    # is the reference's arithmetic, bf16x3 its error-compensated stand-in
    others = {}
    if args.config in ("c2", "c3") and not args.no_fp32:
        del wl
        for prec in [p for p in PRECISIONS if p != args.precision]:
            t2 = Timers()
            log(f"secondary precision {prec}")
            wl2 = build_workload(args, dev, rank, world, prec, t2, dist)
            n2 = max(5, args.steps // (5 if prec == "fp32" else 2))
            dt2, med2 = timed_run(wl2, n2, 3, t2, dist, dev)
            ms2 = dt2 / n2 * 1e3
            others[prec] = {"value": round(samples_per_step * world * n2 / dt2, 1), "unit": "ray-samples/s",
                            "ms_per_step": round(ms2, 3), "ms_per_step_median": round(med2, 3),
                            "steps": n2, "dtype": dtype_of(prec), "precision": prec,
                            "precision_note": PRECISION_NOTE[prec],
                            "roofline": roofline(args, t2, samples_per_step, ms2,
                                                 wl2["core"].step_impl.overlap_dw, precision=prec, steps=n2)}
            del wl2
        clock["after_secondary"] = clock_probe(dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_threads, args)

    if rank == 0:
        metric = {"c2": "ray-samples/sec (train step), SRN-cars 128x128, 64 coarse + 64 fine samples",
                  "c4": "ray-samples/sec (optimize.py code optimisation step), 50 views x 128x128 x 64 samples",
                  "c4eval": "ray-samples/sec (optimize.py evaluation: forward-only render + MSE), 128x128 x 64 samples per view",
                  "c3": "ray-samples/sec (train step), SRN-chairs geometry 128x128, 64 coarse + 64 fine samples",
                  "c5": "ray-samples/sec (train step), SRN-cars 256x256, 128 coarse + 128 fine samples, fp32"}
        out = {
            "metric": metric[args.config],
            "value": round(value, 1), "unit": "ray-samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "ms_per_step_median": round(median, 3),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype_of(args.precision),
            "data": f"synthetic ({H}x{H} ray-cast ellipsoid object per rank, poses on a radius-{radius} sphere, "
                    + (f"trained weights {os.path.relpath(weights_path(args), REPO)})" if weights_path(args)
                       else "random-init weights)"),
            "config": {"workload": f"{'srnchair' if args.config == 'c3' else 'srncar'}.json net, {H}x{H} image/object/step, {args.n_coarse}+{args.n_fine} "
                                   f"samples/ray, " + {"c4": "50 views, codes-only fwd+dX+AdamW",
                                                       "c4eval": "one held-out view per step, forward-only + MSE"}.get(
                                       args.config, "train step incl. AdamW"),
                       "name": args.config, "precision": args.precision,
                       "precision_note": PRECISION_NOTE[args.precision], "objects_per_step": world,
                       "rays_per_step_per_gpu": R, "parallelism": f"dp{world}"},
            "roofline": roof,
            "clock": dict(clock, note=CLOCK_NOTE),
            "precisions": others or None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


CLOCK_NOTE = ("effective shader clock of this box under a dense bf16 MFMA load (cn_clock_probe: every CU, "
              "back-to-back v_mfma_f32_32x32x16_bf16 on hashed operands, s_memtime / s_memrealtime stamps, median "
              "over workgroups; the last of 8 back-to-back ~3 ms launches), measured before the warm-up, after "
              "the timed steps and after the secondary precisions: step times of two runs compare at these clocks")


def clock_probe(dev, n_wg=1024, iters=12000, reps=8):
    """cn_clock_probe on ``dev``, ``reps`` launches back to back (~3 ms each,
    so the clock settles under the load): {"ghz", "ghz_first", "bf16_tflops",
    "ms"} -- the last launch's median over workgroups of stamped shader cycles
    / 100 MHz ticks (and the first launch's), its MFMA rate (n_wg x 4 waves x
    iters x 4 MFMAs x 32,768 FLOP / its wall time) and that wall time."""
    import numpy as np
    from codenerf_amd import _lib
    L = _lib.lib()
    out = torch.zeros(reps, 3 * n_wg, dtype=torch.int32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for r in range(reps):
        _lib.check(L.cn_clock_probe(_lib.ptr(out[r]), n_wg, iters, 12345 + r, _lib.stream_ptr(dev)), "cn_clock_probe")
        ev[r + 1].record()
    torch.cuda.synchronize(dev)
    o = out.cpu().numpy().view(np.uint32).reshape(reps, -1, 3).astype(np.float64)
    ghz = [float(np.median(o[r, :, 0] / np.maximum(o[r, :, 1], 1))) * 0.1 for r in range(reps)]
    ms = ev[reps - 1].elapsed_time(ev[reps])
    tf = n_wg * 4 * iters * 4 * 32768 / (ms * 1e-3) / 1e12
    return {"ghz": round(ghz[-1], 4), "ghz_first": round(ghz[0], 4), "bf16_tflops": round(tf, 1), "ms": round(ms, 3)}


def kernel_roofline(k, precision, timers, traffic):
    """One kernel class against ITS bound, from its launches that ran alone
    (HIP events on the launching stream; launches that shared the chip with
    the other stream's kernel are reported apart under ``contended``):
      fwd / bwd chains -- MFMA-bound: algorithmic FLOPs / time vs the dense
        MFMA peak of the precision;
      dw -- bf16 / bf16x3: HBM-bound, the operand-plane bytes it must read /
        time vs 8 TB/s (its MFMA fraction alongside); fp32: MFMA-bound."""
    peak_tf = FP32_PEAK_TFLOPS if precision == "fp32" else BF16_PEAK_TFLOPS
    t, n, nl = timers.split(k, False)
    basis = f"{nl} uncontended launches, HIP events recorded by each launch's dispatch (hipExtLaunchKernel)"
    if n <= 0 or t <= 0:
        t, n, nl = timers.split(k, True)
        basis = f"{nl} launches beside the other stream's kernel (none ran alone)"
    if n <= 0 or t <= 0:
        return None
    sec = t * 1e-3
    tf = (FLOP_PER_SAMPLE[k] * n + (DW_FOLD_FLOP * nl if k == "dw" else 0)) / sec / 1e12
    out = {"kernel": KERNEL_NAMES[k], "ms_per_launch": round(t / nl, 4), "samples_per_launch": n // nl,
           "basis": basis}
    if k == "dw" and precision != "fp32":
        gbs = DW_BYTES_PER_SAMPLE[precision] * n / sec / 1e9
        out.update(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                   frac=round(gbs / HBM_PEAK_GBS, 4), bytes_per_sample=DW_BYTES_PER_SAMPLE[precision],
                   mfma={"achieved": round(tf, 2), "peak": peak_tf, "unit": "TFLOP/s",
                         "frac": round(tf / peak_tf, 4)})
    elif k == "dw":
        # the exact-fp32 dW pass is MFMA-bound (16 K SIMD cycles of
        # v_mfma_f32_32x32x2_f32 per 64 KiB slab): FLOPs first, bytes beside
        gbs = DW_BYTES_PER_SAMPLE["fp32"] * n / sec / 1e9
        out.update(bound="mfma", achieved=round(tf, 2), peak=peak_tf, unit="TFLOP/s", frac=round(tf / peak_tf, 4),
                   flop_per_sample=FLOP_PER_SAMPLE[k],
                   hbm={"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_sample": DW_BYTES_PER_SAMPLE["fp32"]})
    else:
        out.update(bound="mfma", achieved=round(tf, 2), peak=peak_tf, unit="TFLOP/s", frac=round(tf / peak_tf, 4),
                   flop_per_sample=FLOP_PER_SAMPLE[k])
        if precision == "bf16x3" or (precision == "bf16x3f" and k == "fwd"):
            # three bf16 MFMAs per algorithmic block: the matrix cores' own load
            out["mfma_issued"] = {"achieved": round(3 * tf, 2), "frac": round(3 * tf / peak_tf, 4),
                                  "note": "3 bf16 MFMAs (hi*hi, hi*lo, lo*hi) per algorithmic MFMA"}
    out["traffic"] = traffic
    t_ov, n_ov, l_ov = timers.split(k, True)
    if n_ov > 0 and t_ov > 0 and "beside" not in basis:
        out["contended"] = {"ms_per_launch": round(t_ov / l_ov, 4), "launches": l_ov,
                            "note": "launches overlapped with the other stream's kernel"}
    return out


def roofline(args, timers, samples_per_step, ms, overlapped, precision=None, steps=None):
    """Per-kernel rooflines (fwd and dX chains: MFMA; dW: HBM) and the
    dominant kernel -- the class with the most measured time per step --
    lifted to the top level (bound / achieved / peak / unit / frac / traffic).
    precision / steps: those of this timed run (default: the headline's)."""
    precision = precision or args.precision
    steps = steps or args.steps
    summ = timers.summary()
    if not summ:
        return None
    per_step = {k: v[1] / steps for k, v in summ.items()}    # ms per step (all launches)
    launches = {k: len(timers.ev[k]) / steps for k in timers.ev}
    passes = {"c4": ("fwd", "bwd"), "c4eval": ("fwd",)}.get(args.config, ("fwd", "bwd", "dw"))
    kinds = [k for k in FLOP_PER_SAMPLE if k in summ and k in passes]
    kernels = {}
    for k in kinds:
        r = kernel_roofline(k, precision, timers, load_traffic(args.config, k, precision))
        if r is not None:
            if args.config == "c4eval":
                r["kernel"] = "chain_kernel<fwd,infer>"
            elif args.config == "c4":
                r["kernel"] = {"fwd": "chain_kernel<fwd,codes>", "bwd": "chain_kernel<bwd,codes>"}[k]
            r["launches_per_step"] = launches[k]
            r["ms_per_step"] = round(per_step[k], 4)
            kernels[k] = r
    if not kernels:
        return None
    dom = max(kernels, key=lambda k: per_step[k])
    d = kernels[dom]
    roof = {"bound": d["bound"], "kernel": d["kernel"], "achieved": d["achieved"], "peak": d["peak"],
            "unit": d["unit"], "frac": d["frac"], "traffic": d["traffic"], "basis": d["basis"],
            "ms_per_launch_uncontended": d["ms_per_launch"], "kernels": kernels}
    if overlapped and "dw" in passes:
        roof["overlap"] = ("dX chain of row range i on the main stream || dW of range i-1 on a side stream; "
                           "per-kernel spans overlap, so their sum exceeds the step")
    peak = FP32_PEAK_TFLOPS if precision == "fp32" else BF16_PEAK_TFLOPS
    # SURVEY.md 8(d)'s algorithmic view of the dominant kernel, beside the
    # operand-byte / counter-byte view above: its algorithmic FLOPs against
    # the MFMA peak, and its counted HBM bytes against the step's algorithmic
    # bytes (24 B ray + 12 B gt + 12 B rgb out per ray, spread over the ray's
    # samples) for the samples one launch processes
    alg_tf = d["mfma"]["achieved"] if d["bound"] == "hbm" else d["achieved"]
    n_per_ray = args.n_coarse + args.n_fine
    alg_b = ALG_BYTES_PER_RAY / n_per_ray
    roof["algorithmic"] = {"mfma_achieved": alg_tf, "mfma_peak": peak, "unit": "TFLOP/s",
                           "mfma_frac": round(alg_tf / peak, 4), "hbm_bytes_per_sample": round(alg_b, 4)}
    tr = d.get("traffic")
    if tr:
        alg_launch = alg_b * d["samples_per_launch"]
        roof["algorithmic"].update(hbm_bytes_per_launch=round(alg_launch),
                                   counter_over_algorithmic_bytes=round(tr["hbm_bytes_per_launch"] / alg_launch, 1),
                                   note="the step's own I/O bytes (ray, gt, rgb); the training chains' counted "
                                        "bytes are the activation planes the dW pass reads back (forward: "
                                        "written, dX: read and written) and the weight stream")
    step_flops = sum(v for k, v in FLOP_PER_SAMPLE.items() if k in passes) * samples_per_step
    roof["step"] = {"achieved": round(step_flops / (ms * 1e-3) / 1e12, 2), "unit": "TFLOP/s",
                    "frac": round(step_flops / (ms * 1e-3) / 1e12 / peak, 4)}
    return roof


def load_traffic(config, kernel, precision="bf16"):
    """HBM bytes per launch of a kernel class from the committed rocprofv3
    PMC summary of the same config and precision (profiles/pmc_traffic.json:
    FETCH_SIZE + WRITE_SIZE passes, per launch), or None."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    key = config if precision == "bf16" else f"{config}_{precision}"
    try:
        with open(path) as f:
            t = json.load(f).get(key, {}).get(kernel)
    except OSError:
        return None
    return None if t is None else {"hbm_bytes_per_launch": t["hbm_bytes"], "source": t["source"]}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_quota():
    """CPUs the cgroup grants this process (cpu.max quota / period), or None"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        return None


def cpu_baseline(threads, args):
    """The oracle sample below at the thread counts this process may use: its
    OMP_NUM_THREADS share (16 on the GPU box), the cgroup CPU quota and the
    CPUs it may run on (sched_getaffinity), each at most min(quota,
    affinity).  ``host_cpus`` (os.cpu_count()) is the machine's count, which
    the process is NOT granted on the box (256 CPUs under a 16-CPU quota) and
    is not run.  Each count runs in a child process with a wall-clock limit;
    a count that does not finish is listed as such.  ``value`` / ``cores`` are
    the fastest finished count, every count under ``by_threads``."""
    if threads is not None:
        return _cpu_baseline_at(threads, args, 10.0)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0")) or None
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    quota = cpu_quota()
    # only counts the process may actually use: a thread count above the
    # cgroup quota / affinity (the box: 256 host CPUs on a 16-CPU share)
    # measures oversubscription, not the CPU
    usable = min([c for c in (quota, aff) if c] or [os.cpu_count() or 1])
    counts = sorted({c for c in (omp, quota, aff) if c and c <= usable} or {usable})
    runs, by = [], {}
    for c in counts:
        log(f"cpu baseline, {c} threads (child process, limit 90 s)")
        r = _cpu_baseline_child(c, args, 8.0 if len(counts) > 1 else 10.0, 90)
        if r is None:
            by[c] = "did not finish 2 reps within 90 s"
        else:
            runs.append(r)
            by[c] = r["value"]
    if not runs:
        return None
    best = dict(max(runs, key=lambda r: r["value"]))
    best["by_threads"] = by
    best["affinity_cpus"] = aff
    best["cgroup_cpu_quota"] = quota
    best["usable_cpus"] = usable
    best["omp_num_threads"] = omp
    return best


def _cpu_baseline_child(threads, args, seconds, limit):
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", str(threads),
           "--config", args.config, "--n-coarse", str(args.n_coarse), "--n-fine", str(args.n_fine),
           "--objects", str(args.objects), "--cpu-seconds", str(seconds)]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    try:
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=limit)
    except subprocess.TimeoutExpired:
        return None
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    return json.loads(lines[-1]) if out.returncode == 0 and lines else None


def _cpu_baseline_at(threads, args, seconds):
    """The CPU oracle (torch fp32 restatement of the reference, pinned to its
    golden vectors) on a bounded sample of the SAME step: 1024 rays x
    (n_coarse stratified + n_fine importance) samples -- coarse forward,
    sample_pdf, fine forward, merged composite, both chunk-mean MSEs + code
    regulariser, backward -- then AdamW over the model and both code tables
    (codes-only for c4), timed on this host's cores for ~10 s."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle import ref_cpu
    from oracle.params import make_params
    torch.set_num_threads(threads)
    p = ref_cpu.param_tensors(make_params(0))
    n_obj = args.objects
    st = (torch.randn(n_obj, 256) / 11.3).requires_grad_()
    tt = (torch.randn(n_obj, 256) / 11.3).requires_grad_()
    B, Nc, Nf = 1024, args.n_coarse, args.n_fine
    ro = torch.zeros(B, 3) + torch.tensor([0.0, 0.4, 1.2])
    vd = torch.nn.functional.normalize(torch.randn(B, 3) * 0.2 + torch.tensor([0., -0.3, -1.]), dim=-1)
    z = ref_cpu.stratified_z(0.8, 1.8, Nc)
    gt = torch.rand(B, 3)
    codes_only = args.config == "c4"
    eval_only = args.config == "c4eval"
    groups = [([st], 1e-3), ([tt], 1e-3)] if codes_only else [(list(p.values()), 1e-4), ([st], 1e-3), ([tt], 1e-3)]
    opt = ref_cpu.AdamWRef(groups)

    def one():
        for t in list(p.values()) + [st, tt]:
            t.grad = None
        if eval_only:
            with torch.no_grad():
                xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
                sig, rgbs = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, Nc, -1), st[0][None], tt[0][None])
                rgb, _ = ref_cpu.volume_rendering(sig, rgbs, z)
                ((rgb - gt) ** 2).mean()
            return
        if Nf:
            with torch.no_grad():
                xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
                sig_c, _ = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, Nc, -1), st[0][None], tt[0][None])
                z_f = ref_cpu.sample_pdf(sig_c[..., 0], z, torch.rand(B, Nf))
            ref_cpu.fine_image_step(p, st, tt, 0, ro, vd, z, z_f, gt, chunk=B)
        else:
            ref_cpu.image_step(p, st, tt, 0, ro, vd, z, gt, chunk=B)
        opt.step()

    one()
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds or reps < 2:
        one()
        reps += 1
    dt = time.perf_counter() - t0
    what = "forward + composite + MSE (no grad)" if eval_only else \
        "codes-only fwd+composite+MSE+backward+AdamW(codes)" if codes_only else \
        ("coarse fwd + sample_pdf + fine fwd + merged composite + MSEs + backward + AdamW(model, code tables)"
         if Nf else "fwd+composite+MSE+backward+AdamW")
    return {"value": round(B * (Nc + Nf) * reps / dt, 1), "unit": "ray-samples/s", "cores": threads,
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model(), "kind": "port",
            "sample": f"{reps} x ({B} rays x {Nc}+{Nf} samples) {what}, torch CPU fp32 oracle "
                      f"(oracle/ref_cpu.py" + ("; the coarse forward runs twice, once without grad for sample_pdf" if Nf else "")
                      + f"), {threads} threads"}


if __name__ == "__main__":
    main()
