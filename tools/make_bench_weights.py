"""Trained weights for bench.py --weights (verdict r3 item 4: the bench ran
on random-init weights only, and the chain kernels' time depends on their
inputs through the chip's clock).

Trains the srncar net through the reference loop (codenerf_amd.trainer.Trainer
= src/trainer.py:34-101: AdamW re-created per epoch, srncar.json learning
rates) on N_OBJ synthetic SRN-format cars at the bench's C2 geometry (128^2
views, focal 131.25, near / far 0.8 / 1.8, 64 coarse + 64 fine samples) in
fp32 for ITERS steps, and writes the reference checkpoint format (models.pth:
model_params / shape_code_params / texture_code_params) to
weights/c2_regime_<ITERS>.pth.

  python tools/make_bench_weights.py [iters] [n_obj]      (GPU)
"""
import os
import shutil
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    n_obj = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    from codenerf_amd.data import make_synthetic_srn
    from codenerf_amd.trainer import Trainer
    tmp = tempfile.mkdtemp()
    root = os.path.join(tmp, "data")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=n_obj, n_views=4, H=128, W=128, focal=131.25, seed=5)
    hp = {"net_hyperparams": {"shape_blocks": 3, "texture_blocks": 1, "W": 256, "num_xyz_freq": 10,
                              "num_dir_freq": 4, "latent_dim": 256},
          "data": {"cat": "srn_cars", "splits": "cars_train", "data_dir": root, "n_train_views": 4},
          "N_samples": 64, "N_importance": 64, "near": 0.8, "far": 1.8, "loss_reg_coef": 1e-4,
          "lr_schedule": [{"type": "step", "lr": 1e-4, "interval": 250000},
                          {"type": "step", "lr": 1e-3, "interval": 250000}],
          "check_points": 10 ** 9, "precision": "fp32"}
    torch.manual_seed(0)
    np.random.seed(0)
    tr = Trainer("bench_weights", 0, hpams=hp, batch_size=2048, check_iter=0, exp_root=os.path.join(tmp, "exps"))
    tr.training(0, iters, 1)
    ps = np.array(tr.psnr_log)
    print(f"train PSNR: first epoch {ps[:n_obj].mean():.2f} dB, last epoch {ps[-n_obj:].mean():.2f} dB "
          f"over {len(ps)} steps", flush=True)
    os.makedirs(os.path.join(REPO, "weights"), exist_ok=True)
    dst = os.path.join(REPO, "weights", f"c2_regime_{iters}.pth")
    shutil.copy(os.path.join(tr.save_dir, "models.pth"), dst)
    print("wrote", dst)


if __name__ == "__main__":
    main()
