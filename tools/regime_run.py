"""One HIP training trajectory of tests/test_gpu_regime.py's many-object
regime (8 synthetic cars, 64^2, 64 samples, AdamW re-created per epoch,
srncar.json rates) -> per-step train PSNR in an .npz.  Used to compare
library builds / precisions over several seeds (one process per run: the
library is loaded once per process; CODENERF_LIB + CODENERF_MEASURE=1 select a
measurement build).

  python tools/regime_run.py OUT.npz PRECISION SEED [EPOCHS] [--no-overlap] [--fine N]
"""
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    out, prec, seed = sys.argv[1], sys.argv[2], int(sys.argv[3])
    epochs = int(sys.argv[4]) if len(sys.argv) > 4 and not sys.argv[4].startswith("--") else 40
    overlap = "--no-overlap" not in sys.argv
    fine = int(sys.argv[sys.argv.index("--fine") + 1]) if "--fine" in sys.argv else 0
    from codenerf_amd.data import make_synthetic_srn
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.trainer import Trainer
    from test_gpu_regime import hp_many, N_OBJ, H, FOCAL
    tmp = tempfile.mkdtemp()
    root = os.path.join(tmp, "data")
    make_synthetic_srn(root, "srn_cars", "cars_train", n_obj=N_OBJ, n_views=2, H=H, W=H, focal=FOCAL, seed=21)
    hp = hp_many(root, prec)
    hp["N_importance"] = fine
    # identical initial weights for every precision / build of a seed: the
    # Trainer's own init sequence on the CPU generator, then loaded
    torch.manual_seed(seed)
    np.random.seed(seed)
    tr = Trainer(f"rr_{prec}_{seed}", 0, hpams=hp, batch_size=2048, check_iter=0, exp_root=os.path.join(tmp, "exps"))
    tr.step_impl.overlap_dw = overlap
    torch.manual_seed(1000 + seed)
    np.random.seed(1000 + seed)
    tr.training(0, epochs * N_OBJ, 1)
    np.savez(out, psnr=np.array(tr.psnr_log), prec=prec, seed=seed, overlap=overlap,
             lib=os.environ.get("CODENERF_LIB", "in-tree"))
    print(out, prec, seed, overlap, np.round(np.array(tr.psnr_log)[-8:], 3).tolist(), flush=True)


if __name__ == "__main__":
    main()
