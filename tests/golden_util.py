"""Helpers shared by the oracle and GPU parity tests (test infrastructure)."""
import os

import numpy as np
import torch

from oracle import ref_cpu
from oracle.params import make_params

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

TRAIN_CASES = ["c1_32x32_n32", "dense_16x16_n32", "n64_16x16", "n96_16x16_chairs",
               "n128_8x8", "chunks_64x64_n16", "ragged_48x48_n16"]


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def case_params(g):
    return make_params(int(g["seed"]), sigma_bias_shift=float(g["sigma_shift"]))


def digest_matches(g, key, arr, rtol=2e-4, atol=1e-7, scale_tol=1e-4):
    """Compare a tensor with the digest stored under grad/<key>/... ."""
    a = np.asarray(arr, dtype=np.float64).reshape(-1)
    idx = g[f"grad/{key}/idx"]
    vals = g[f"grad/{key}/vals"].astype(np.float64)
    scale = max(np.abs(vals).max(), 1e-12)
    ok_vals = np.allclose(a[idx], vals, rtol=rtol, atol=atol + scale_tol * scale)
    s, ss = float(g[f"grad/{key}/sum"]), float(g[f"grad/{key}/sumsq"])
    ok_ss = abs(float((a * a).sum()) - ss) <= max(rtol * 10, 4 * scale_tol) * abs(ss) + 1e-20
    ok_sum = abs(float(a.sum()) - s) <= 1e-3 * np.sqrt(ss * a.size) + 1e-12
    return ok_vals and ok_ss and ok_sum, (a[idx] - vals).__abs__().max()


def oracle_image_step(g, chunk=None, reg_coef=1e-4):
    """Replays one training image with the CPU oracle; returns dict of results."""
    p = ref_cpu.param_tensors(case_params(g))
    st = torch.tensor(g["shape_table"], requires_grad=True)
    tt = torch.tensor(g["texture_table"], requires_grad=True)
    ro, vd = torch.tensor(g["rays_o"]), torch.tensor(g["viewdir"])
    z = torch.tensor(g["z_vals"])
    gt = torch.tensor(g["gt"])
    losses, rgb = ref_cpu.image_step(p, st, tt, int(g["obj_idx"]), ro, vd, z, gt,
                                     chunk=int(g["chunk"]) if chunk is None else chunk,
                                     reg_coef=reg_coef)
    return dict(params=p, shape_table=st, texture_table=tt, losses=losses, rgb=rgb)


def oracle64_image_step(g):
    """The oracle replayed in float64: ground truth for fp32 error budgets."""
    p = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in case_params(g).items()}
    st = torch.tensor(g["shape_table"], dtype=torch.float64, requires_grad=True)
    tt = torch.tensor(g["texture_table"], dtype=torch.float64, requires_grad=True)
    f = lambda k: torch.tensor(g[k], dtype=torch.float64)
    losses, rgb = ref_cpu.image_step(p, st, tt, int(g["obj_idx"]), f("rays_o"), f("viewdir"), f("z_vals"),
                                     f("gt"), chunk=int(g["chunk"]))
    return dict(params=p, shape_table=st, texture_table=tt, losses=losses, rgb=rgb)


def rel_err(a, b):
    """max |a - b| / max |b| (b: the more accurate value)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))
