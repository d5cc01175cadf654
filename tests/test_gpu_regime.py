"""GPU: train PSNR in the reference's own optimiser regime.

The reference trains MANY objects per epoch and re-creates AdamW only at the
start of an epoch (src/trainer.py:48-96, :52), so Adam's moments persist
across the n_obj steps of an epoch; its learning rates are srncar.json's
(1e-4 model, 1e-3 codes).  This test runs that regime -- N_OBJ synthetic
SRN-format objects, H x H views, N samples per ray, EPOCHS epochs -- from
identical initial weights and RNG draws through:

  * the HIP trainer in fp32 (the reference precision),
  * the HIP trainer in bf16 (BASELINE C2's operand precision),
  * the HIP trainer in bf16s (error-compensated: weights carried as
    bf16 hi + lo pairs, two MFMAs per block into one fp32 accumulator),
  * the fp32 CPU replay of the reference loop (oracle/ref_cpu.py),

and asserts each one's per-step train PSNR (src/trainer.py:98-101) against the
fp32 replay.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_OBJ, H, N, EPOCHS = 8, 64, 64, 4
FOCAL = 65.625              # SRN-cars focal (131.25 at 128^2) scaled to H
B = 2048                    # rays per loss chunk (src/trainer.py:69)


def hp_many(root, prec):
    return {"net_hyperparams": {"shape_blocks": 3, "texture_blocks": 1, "W": 256, "num_xyz_freq": 10,
                                "num_dir_freq": 4, "latent_dim": 256},
            "data": {"cat": "srn_cars", "splits": "cars_train", "data_dir": root, "n_train_views": 2},
            "N_samples": N, "near": 0.8, "far": 1.8, "loss_reg_coef": 1e-4,
            "lr_schedule": [{"type": "step", "lr": 1e-4, "interval": 250000},
                            {"type": "step", "lr": 1e-3, "interval": 250000}],
            "check_points": 10 ** 9, "N_importance": 0, "precision": prec}

REPLAY_STEPS = 2 * N_OBJ    # CPU replay horizon (two epochs; ~3 s per 262K-sample step on 16 threads)
LONG_EPOCHS = 40            # HIP-only horizon: every precision against HIP fp32


def _data(tmp_path):
    from codenerf_amd.data import make_synthetic_srn
    root = str(tmp_path / "data")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=N_OBJ, n_views=2, H=H, W=H, focal=FOCAL, seed=21)
    return root


def _run(tmp_path, root, prec, iters, init=None, seed=0):
    from codenerf_amd.trainer import Trainer
    torch.manual_seed(seed)
    np.random.seed(seed)
    tr = Trainer(f"r_{prec}_{iters}", 0, hpams=hp_many(root, prec), batch_size=B, check_iter=0,
                 exp_root=str(tmp_path / "exps"))
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
    tr.training(0, iters, 1)
    return np.array(tr.psnr_log), init


@pytest.mark.timeout(900)
def test_many_objects_train_psnr_vs_fp32_replay(tmp_path):
    """Every precision's per-step train PSNR within 0.05 dB of the fp32 CPU
    replay over the replay horizon (two epochs of N_OBJ objects)."""
    import os
    from test_gpu_train import _oracle_training
    root = _data(tmp_path)
    runs = {}
    runs["fp32"], init = _run(tmp_path, root, "fp32", REPLAY_STEPS)
    for prec in ("bf16", "bf16x3"):
        runs[prec], _ = _run(tmp_path, root, prec, REPLAY_STEPS, init)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    torch.manual_seed(1000)
    np.random.seed(1000)
    ref, _, _, _ = _oracle_training(hp_many(root, "fp32"), init, REPLAY_STEPS, B)
    ref = np.array(ref)
    print(f"\nfp32 replay   {np.round(ref, 3).tolist()}")
    for prec, r in runs.items():
        print(f"HIP {prec:7s}  {np.round(r, 3).tolist()}  max |d| vs replay {np.abs(r - ref).max():.4f} dB")
    for prec, r in runs.items():
        assert np.abs(r - ref).max() <= 0.05, prec


@pytest.mark.timeout(900)
def test_many_objects_long_horizon_vs_fp32(tmp_path):
    """LONG_EPOCHS epochs (the CPU replay would take hours): bf16x3 and bf16
    against HIP fp32 -- which follows the fp32 replay, previous test -- on
    the last epoch's mean train PSNR and per step."""
    root = _data(tmp_path)
    iters = LONG_EPOCHS * N_OBJ
    runs = {}
    runs["fp32"], init = _run(tmp_path, root, "fp32", iters)
    for prec in ("bf16", "bf16x3"):
        runs[prec], _ = _run(tmp_path, root, prec, iters, init)
    last = {k: float(v[-N_OBJ:].mean()) for k, v in runs.items()}
    d = {k: np.abs(v - runs["fp32"]) for k, v in runs.items()}
    print(f"\nlast-epoch mean train PSNR {last}; first epoch {runs['fp32'][:N_OBJ].mean():.3f} dB (fp32)")
    for k in ("bf16", "bf16x3"):
        print(f"{k}: last-epoch gap {last[k] - last['fp32']:+.4f} dB, per-step max |d| {d[k].max():.4f} dB")
    assert last["fp32"] > runs["fp32"][:N_OBJ].mean() + 3.0        # the run is learning
    for k in ("bf16", "bf16x3"):
        assert abs(last[k] - last["fp32"]) <= 0.05, k
