"""More seeds of tests/test_gpu_regime.py's long-horizon measurement (the
reference's many-object regime, 40 epochs): per seed, the epoch at which HIP
fp32 / bf16x3 / bf16 first leave 0.05 dB of the reference loop replayed in
torch fp32 on the GPU, and the horizon where HIP fp32 stays within 0.025 dB
of it.  A record for DESIGN.md, not a test.

  python tools/regime_seeds.py OUT.json SEED [SEED ...]
"""
import json
import os
import sys
import tempfile
import pathlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import test_gpu_regime as R
    out, seeds = sys.argv[1], [int(s) for s in sys.argv[2:]]
    tmp = pathlib.Path(tempfile.mkdtemp())
    root = R._data(tmp)
    iters = R.LONG_EPOCHS * R.N_OBJ
    rows = []
    for seed in seeds:
        runs = {}
        runs["fp32"], init = R._run(tmp, root, "fp32", iters, seed=seed)
        for prec in ("bf16", "bf16x3"):
            runs[prec], _ = R._run(tmp, root, prec, iters, init, seed=seed)
        runs["ref"] = R.reference_on_gpu(root, init, iters, seed, R.hp_many(root, "fp32"))
        em = {k: R._epoch_means(v) for k, v in runs.items()}
        horizon, gap = R.horizon_report("coarse", seed, em, R.LONG_EPOCHS)
        rows.append({"seed": seed, "horizon": horizon,
                     "first_exit": {k: R.first_exit(g) for k, g in gap.items()},
                     "max_gap_within_horizon": {k: round(float(g[:horizon].max()), 4) for k, g in gap.items()}})
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
