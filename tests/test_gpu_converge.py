"""GPU: a CONVERGING train-PSNR trajectory (BASELINE metric "train PSNR";
north_star "PSNR within 0.05 dB of reference").

One synthetic SRN-format object (one 32x32 view), the reference loop
(src/trainer.py:34-96: AdamW re-created every epoch -- with one object every
step --, zero_grad inside the image loop, chunk-mean MSE + code regulariser,
LR halving) with a faster LR schedule than srncar.json's so the run crosses
20 dB within the test's budget.  Three trajectories from the same initial
weights, data and RNG draws:

  * the fp32 CPU replay of the reference loop (oracle), affordable for the
    first REPLAY steps;
  * the HIP fp32 trainer, all ITERS steps;
  * the HIP bf16 trainer (the benchmarked precision), all ITERS steps.

Checked: the run converges (fp32 PSNR > 20 dB at the end); HIP fp32 follows
the CPU replay within 0.01 dB over the replayed prefix and bf16 within
0.05 dB; at the end the bf16 trajectory is within 0.05 dB of the fp32 one
(mean over the last 50 steps).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ITERS, REPLAY = 600, 60


def _hp(root, prec):
    return {"net_hyperparams": {"shape_blocks": 3, "texture_blocks": 1, "W": 256, "num_xyz_freq": 10,
                                "num_dir_freq": 4, "latent_dim": 256},
            "data": {"cat": "srn_cars", "splits": "cars_train", "data_dir": root, "n_train_views": 1},
            "N_samples": 32, "near": 0.8, "far": 1.8, "loss_reg_coef": 1e-4,
            "lr_schedule": [{"type": "step", "lr": 1e-3, "interval": 100},
                            {"type": "step", "lr": 1e-2, "interval": 100}],
            "check_points": 10 ** 9, "N_importance": 0, "precision": prec}


@pytest.mark.timeout(600)
def test_converging_train_psnr_bf16_matches_fp32(tmp_path):
    from codenerf_amd.data import make_synthetic_srn
    from codenerf_amd.trainer import Trainer
    from test_gpu_train import _oracle_training
    root = str(tmp_path / "data")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=1, n_views=1, H=32, W=32, focal=32.8, seed=11)
    runs, init = {}, None
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        np.random.seed(0)
        tr = Trainer("c_" + prec, 0, hpams=_hp(root, prec), batch_size=256, check_iter=0,
                     exp_root=str(tmp_path / "exps"))
        if init is None:
            init = {"model": {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()},
                    "shape": tr.shape_codes.weight.detach().cpu().clone(),
                    "texture": tr.texture_codes.weight.detach().cpu().clone()}
        else:       # same initial weights and codes for both precisions
            tr.model.load_state_dict(init["model"])
            with torch.no_grad():
                tr.shape_codes.weight.copy_(init["shape"])
                tr.texture_codes.weight.copy_(init["texture"])
        torch.manual_seed(1)
        np.random.seed(1)
        tr.training(0, ITERS, 1)
        runs[prec] = np.array(tr.psnr_log)
    torch.manual_seed(1)
    np.random.seed(1)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref, _, _, _ = _oracle_training(_hp(root, "fp32"), init, REPLAY, 256)
    ref = np.array(ref)
    p32, p16 = runs["fp32"], runs["bf16"]
    d32 = np.abs(p32[:REPLAY] - ref)
    d16 = np.abs(p16[:REPLAY] - ref)
    tail = abs(p16[-50:].mean() - p32[-50:].mean())
    print(f"\nfinal PSNR fp32 {p32[-1]:.3f} bf16 {p16[-1]:.3f}; last-50 mean fp32 {p32[-50:].mean():.3f} "
          f"bf16 {p16[-50:].mean():.3f} (|d| {tail:.4f} dB); replay prefix max|d| fp32 {d32.max():.4f} "
          f"bf16 {d16.max():.4f} dB; first > 20 dB: fp32 {int(np.argmax(p32 > 20))} bf16 {int(np.argmax(p16 > 20))}")
    print("every 25th step fp32:", np.round(p32[::25], 2).tolist())
    print("every 25th step bf16:", np.round(p16[::25], 2).tolist())
    assert p32[-50:].mean() > 20.0 and p16[-50:].mean() > 20.0
    assert d32.max() <= 0.01
    assert d16.max() <= 0.05
    assert tail <= 0.05
