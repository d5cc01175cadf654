"""GPU probe: train-PSNR trajectories of the reference loop (codenerf_amd.trainer)
on one synthetic object under several learning-rate schedules, to pick the
schedule of tests/test_gpu_converge.py.

  python tools/converge_probe.py <iters> <prec> <lr_model>,<lr_code>,<interval> ...
"""
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from codenerf_amd.data import make_synthetic_srn
    from codenerf_amd.trainer import Trainer
    iters, prec = int(sys.argv[1]), sys.argv[2]
    tmp = tempfile.mkdtemp()
    root = os.path.join(tmp, "data")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=1, n_views=1, H=32, W=32, focal=32.8, seed=11)
    for spec in sys.argv[3:]:
        lm, lc, iv = spec.split(",")
        hp = {"net_hyperparams": {"shape_blocks": 3, "texture_blocks": 1, "W": 256, "num_xyz_freq": 10,
                                  "num_dir_freq": 4, "latent_dim": 256},
              "data": {"cat": "srn_cars", "splits": "cars_train", "data_dir": root, "n_train_views": 1},
              "N_samples": 32, "near": 0.8, "far": 1.8, "loss_reg_coef": 1e-4,
              "lr_schedule": [{"type": "step", "lr": float(lm), "interval": int(iv)},
                              {"type": "step", "lr": float(lc), "interval": int(iv)}],
              "check_points": 10 ** 9, "N_importance": 0, "precision": prec}
        torch.manual_seed(0)
        np.random.seed(0)
        tr = Trainer("p", 0, hpams=hp, batch_size=256, check_iter=0, exp_root=os.path.join(tmp, "exps"))
        tr.training(0, iters, 1)
        ps = tr.psnr_log
        print(spec, [round(ps[i], 2) for i in range(0, iters, max(1, iters // 20))], round(ps[-1], 2),
              "first>20:", next((i for i, p in enumerate(ps) if p > 20), None), flush=True)


if __name__ == "__main__":
    main()
