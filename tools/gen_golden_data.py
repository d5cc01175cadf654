"""Golden vectors for the SRN loader: run the REFERENCE's src/data.py parsing
functions (load_poses, load_intrinsic) on a small synthetic SRN-format split
written by codenerf_amd.data.make_synthetic_srn, and store the parsed arrays.

src/data.py imports imageio at module level; only the parsing helpers that do
not touch it are called, and a stub module satisfies the import (the same
arrangement as tools/gen_golden.py).  Output: tests/golden/srn_loader.npz
(the synthetic split itself is regenerated from its seed by the test).

Usage:  python tools/gen_golden_data.py [--ref /root/reference]
"""
import argparse
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

SPEC = dict(n_obj=2, n_views=3, H=32, W=32, focal=35.0, radius=1.3, seed=11)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    from codenerf_amd.data import make_synthetic_srn
    sys.dont_write_bytecode = True
    if "imageio" not in sys.modules:
        sys.modules["imageio"] = types.ModuleType("imageio")
    sys.path.insert(0, os.path.join(args.ref, "src"))
    import data as ref_data  # noqa
    sys.path.pop(0)
    with tempfile.TemporaryDirectory() as tmp:
        base = make_synthetic_srn(tmp, "srn_cars", "cars_train", **SPEC)
        ids = sorted(os.listdir(base))
        out = {}
        for k, oid in enumerate(ids):
            poses = ref_data.load_poses(os.path.join(base, oid, "pose"), [2, 0, 1])
            focal, H, W = ref_data.load_intrinsic(os.path.join(base, oid, "intrinsics.txt"))
            out[f"poses_{k}"] = poses.numpy()
            out[f"intr_{k}"] = np.array([focal, H, W], dtype=np.float64)
        out["spec"] = np.array([SPEC[k] for k in ("n_obj", "n_views", "H", "W", "focal", "radius", "seed")])
        np.savez_compressed(os.path.join(REPO, "tests", "golden", "srn_loader.npz"), **out)
    print("wrote tests/golden/srn_loader.npz")


if __name__ == "__main__":
    main()
