"""GPU: train PSNR on the BENCHMARKED workload shape -- 64 coarse + 64 fine
samples per ray (BASELINE configs[1]) -- in the reference's optimiser regime.

test_gpu_regime.py runs the regime coarse-only; the bench measures the 64 + 64
step.  Here N_OBJ synthetic SRN-format cars (H x H views, srncar.json
learning rates, AdamW re-created per epoch: src/trainer.py:48-101) train
through the HIP Trainer with N_importance = 64, from identical initial
weights and RNG draws, in fp32, bf16, bf16x3 and bf16x3f, and through the oracle's CPU
replay of the same loop with the fine pass (oracle/ref_cpu.py:
sample_pdf + fine_image_step).  The fine uniforms are the Trainer's own
device draws (torch.rand(R, N_fine) on cuda:0, one per step): the replay
re-seeds the same generator and copies its draws to the host, so both sides
sample from the same uniforms; each side inverts its OWN coarse densities
(the fine pass has no reference -- sample_pdf is NeRF's hierarchical
sampling as this build defines it, parity unpinned; test_gpu_fine.py checks
the kernels against the restatement).

  * replay horizon (REPLAY_STEPS): every precision's per-step fine train
    PSNR (src/trainer.py:98-101 on the fine chunk losses) against the fp32
    CPU replay;
  * long horizon (LONG_EPOCHS): epoch means against the same loop replayed
    in torch fp32 on the GPU, over the horizon where HIP fp32 itself stays
    within half the bar of it (test_gpu_regime.horizon_report).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_OBJ, H, NC, NF = 8, 64, 64, 64
FOCAL = 65.625              # SRN-cars focal (131.25 at 128^2) scaled to H
B = 2048                    # rays per loss chunk (src/trainer.py:69)
REPLAY_STEPS = 2 * N_OBJ    # CPU replay: two epochs (~4 s per 0.5 M-sample step on 16 threads)
LONG_EPOCHS = 40
BAR_DB = 0.05


def hp_fine(root, prec):
    return {"net_hyperparams": {"shape_blocks": 3, "texture_blocks": 1, "W": 256, "num_xyz_freq": 10,
                                "num_dir_freq": 4, "latent_dim": 256},
            "data": {"cat": "srn_cars", "splits": "cars_train", "data_dir": root, "n_train_views": 2},
            "N_samples": NC, "N_importance": NF, "near": 0.8, "far": 1.8, "loss_reg_coef": 1e-4,
            "lr_schedule": [{"type": "step", "lr": 1e-4, "interval": 250000},
                            {"type": "step", "lr": 1e-3, "interval": 250000}],
            "check_points": 10 ** 9, "precision": prec}


def _data(tmp_path, h=H, focal=FOCAL):
    from codenerf_amd.data import make_synthetic_srn
    root = str(tmp_path / f"data{h}")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=N_OBJ, n_views=2, H=h, W=h, focal=focal, seed=21)
    return root


def _run(tmp_path, root, prec, iters, init=None, seed=0, overlap=True):
    from codenerf_amd.trainer import Trainer
    torch.manual_seed(seed)
    np.random.seed(seed)
    tr = Trainer(f"f_{prec}_{iters}_{int(overlap)}", 0, hpams=hp_fine(root, prec), batch_size=B, check_iter=0,
                 exp_root=str(tmp_path / "exps"))
    tr.step_impl.overlap_dw = overlap
    if init is None:
        init = {"model": {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()},
                "shape": tr.shape_codes.weight.detach().cpu().clone(),
                "texture": tr.texture_codes.weight.detach().cpu().clone()}
    else:
        tr.model.load_state_dict(init["model"])
        with torch.no_grad():
            tr.shape_codes.weight.copy_(init["shape"])
            tr.texture_codes.weight.copy_(init["texture"])
    torch.manual_seed(1000 + seed)          # CPU (z jitter) and cuda:0 (fine uniforms) generators
    np.random.seed(1000 + seed)
    tr.training(0, iters, 1)
    return np.array(tr.psnr_log), init


def _oracle_training_fine(hp, init, iters, seed=0, device=None):
    """The CPU replay of src/trainer.py:34-101 with the fine pass: per step
    the z jitter from the host generator (as the Trainer), the fine uniforms
    drawn on cuda:0 exactly as the Trainer draws them and copied to the host,
    the coarse densities of the replay's own no-grad forward -> sample_pdf ->
    fine_image_step; PSNR of the mean fine chunk loss.  ``device`` "cuda":
    the same replay in torch fp32 on the GPU (same random draws)."""
    from codenerf_amd.data import SRN, collate_one
    from oracle import ref_cpu
    dev = torch.device(device) if device is not None else torch.device("cpu")
    p = {k: v.to(dev).clone().requires_grad_() for k, v in init["model"].items()}
    st = init["shape"].to(dev).clone().requires_grad_()
    tt = init["texture"].to(dev).clone().requires_grad_()
    d = hp["data"]
    torch.manual_seed(1000 + seed)
    np.random.seed(1000 + seed)
    psnrs, niter = [], 0
    while niter < iters:
        ds = SRN(d["cat"], d["splits"], d["data_dir"], 1, crop_img=False, n_train_views=d["n_train_views"])
        ms, ls = hp["lr_schedule"]
        opt = ref_cpu.AdamWRef([(list(p.values()), ms["lr"]), ([st], ls["lr"]), ([tt], ls["lr"])])
        for idx in range(len(ds)):
            if niter >= iters:
                break
            focal, Hh, Ww, imgs, poses, _, oi = collate_one(ds[idx])
            for t in list(p.values()) + [st, tt]:
                t.grad = None
            ro, vd = ref_cpu.get_rays(int(Hh), int(Ww), focal, poses[0, 0])
            ro, vd = ro.to(dev), vd.to(dev)
            z = ref_cpu.stratified_z(hp["near"], hp["far"], hp["N_samples"]).to(dev)
            rnd = torch.rand(int(Hh) * int(Ww), hp["N_importance"], device="cuda").to(dev)
            with torch.no_grad():
                xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
                sig_c, _ = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, z.shape[0], -1),
                                                    st[int(oi)][None], tt[int(oi)][None])
                z_f = ref_cpu.sample_pdf(sig_c[..., 0], z, rnd)
            _, lf, _ = ref_cpu.fine_image_step(p, st, tt, int(oi), ro, vd, z, z_f, imgs[0, 0].to(dev), chunk=B,
                                               reg_coef=hp["loss_reg_coef"])
            opt.step()
            psnrs.append(-10 * np.log(np.mean(lf)) / np.log(10))
            niter += 1
    return np.array(psnrs)


@pytest.mark.timeout(900)
def test_fine_regime_train_psnr_vs_fp32_replay(tmp_path):
    """64 + 64 samples: per-step fine train PSNR of HIP fp32 / bf16x3 within
    0.05 dB of the fp32 CPU replay over two epochs; bf16 printed."""
    root = _data(tmp_path)
    runs = {}
    runs["fp32"], init = _run(tmp_path, root, "fp32", REPLAY_STEPS)
    for prec in ("bf16", "bf16x3"):
        runs[prec], _ = _run(tmp_path, root, prec, REPLAY_STEPS, init)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = _oracle_training_fine(hp_fine(root, "fp32"), init, REPLAY_STEPS)
    print(f"\nfp32 replay (64+64)  {np.round(ref, 3).tolist()}")
    gaps = {}
    for prec, r in runs.items():
        gaps[prec] = np.abs(r - ref).max()
        print(f"HIP {prec:7s}  {np.round(r, 3).tolist()}  max |d| vs replay {gaps[prec]:.4f} dB")
    assert gaps["fp32"] <= BAR_DB
    assert gaps["bf16x3"] <= BAR_DB


def _epoch_means(r):
    return r[: len(r) // N_OBJ * N_OBJ].reshape(-1, N_OBJ).mean(1)


@pytest.mark.timeout(900)
def test_fine_regime_long_horizon_vs_reference(tmp_path):
    """LONG_EPOCHS epochs of the 64 + 64 regime for two initialisations: the
    HIP trainer in fp32 / bf16 / bf16x3 against the same loop replayed in
    torch fp32 on the GPU (_oracle_training_fine on cuda:0, the Trainer's own
    fine uniforms), by epoch-mean fine train PSNR.  Asserted: the runs learn
    and the horizon (HIP fp32 within half the bar, horizon_report) leaves a
    meaningful window; whether bf16x3 stays within 0.05 dB over it is
    recorded (PASS, or XFAIL with the exit: test_gpu_regime.trajectory_bar);
    bf16 and bf16x3f printed."""
    from test_gpu_regime import horizon_report, trajectory_bar
    root = _data(tmp_path)
    iters = LONG_EPOCHS * N_OBJ
    per_seed = []
    for seed in (0, 1):
        runs = {}
        runs["fp32"], init = _run(tmp_path, root, "fp32", iters, seed=seed)
        for prec in ("bf16", "bf16x3", "bf16x3f"):
            runs[prec], _ = _run(tmp_path, root, prec, iters, init, seed=seed)
        runs["ref"] = _oracle_training_fine(hp_fine(root, "fp32"), init, iters, seed=seed, device="cuda")
        em = {k: _epoch_means(v) for k, v in runs.items()}
        horizon, gap = horizon_report("fine", seed, em, LONG_EPOCHS)
        assert em["ref"][-1] > em["ref"][0] + 3.0          # the run is learning
        assert horizon >= 10
        per_seed.append((seed, gap, horizon))
    for seed, gap, horizon in per_seed:
        trajectory_bar(f"fine seed {seed}", gap, horizon)


C2_EPOCHS = 32
C2_TAIL = 10


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("seed", [0, 1])
def test_fine_regime_c2_image_size_vs_reference(tmp_path, seed):
    """The benchmarked configuration itself (BASELINE configs[1]: 128 x 128
    views, SRN-cars focal 131.25, 64 + 64 samples) in the reference's
    many-object regime: C2_EPOCHS epochs of N_OBJ objects -- past the 20+
    epochs where two fp32 orders separate at 64^2 -- through the HIP trainer
    in fp32, bf16x3, bf16x3f and bf16 against the same loop replayed in torch
    fp32 on the GPU (_oracle_training_fine, the Trainer's own fine
    uniforms), by epoch-mean fine train PSNR.  Asserted: the run learns and
    the horizon leaves a meaningful window; whether bf16x3 stays within
    0.05 dB of the reference over the horizon where HIP fp32 stays within half
    the bar is recorded (PASS, or XFAIL with the exit:
    test_gpu_regime.trajectory_bar).  Printed: every run's first exit and its
    mean over the last C2_TAIL epochs against the reference's."""
    from test_gpu_regime import horizon_report, trajectory_bar
    root = _data(tmp_path, 128, 131.25)
    iters = C2_EPOCHS * N_OBJ
    runs = {}
    runs["fp32"], init = _run(tmp_path, root, "fp32", iters, seed=seed)
    for prec in ("bf16x3", "bf16x3f", "bf16"):
        runs[prec], _ = _run(tmp_path, root, prec, iters, init, seed=seed)
    runs["ref"] = _oracle_training_fine(hp_fine(root, "fp32"), init, iters, seed=seed, device="cuda")
    em = {k: _epoch_means(v) for k, v in runs.items()}
    horizon, gap = horizon_report("fine 128^2", seed, em, C2_EPOCHS)
    tail = {k: float(v[-C2_TAIL:].mean() - em["ref"][-C2_TAIL:].mean()) for k, v in em.items() if k != "ref"}
    print(f"fine 128^2 seed {seed}: last-{C2_TAIL}-epoch mean minus the reference's: "
          + ", ".join(f"{k} {v:+.4f} dB" for k, v in tail.items()))
    assert em["ref"][-1] > em["ref"][0] + 3.0          # the run is learning
    assert horizon >= 10
    trajectory_bar(f"fine 128^2 seed {seed}", gap, horizon)
