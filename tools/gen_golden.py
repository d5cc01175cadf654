"""Generate golden vectors by running the REFERENCE implementation.

Imports /root/reference/src/model.py and src/utils.py (read-only, bytecode
writing disabled, a stub ``imageio`` module because src/utils.py:2 imports it
but the hot-path functions never use it) and runs the hot path on seeded
inputs.  Only the resulting arrays are written (tests/golden/*.npz); no
reference source or bytecode is copied.  The training-loop body
(src/trainer.py:65-85) cannot be imported (it needs tensorboard), so it is
replayed here line-for-line around the imported model/utils.

Usage:  python tools/gen_golden.py [--ref /root/reference]
"""
import argparse
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from oracle.params import make_params, make_codes, look_at_pose  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")


def import_reference(ref_root):
    sys.dont_write_bytecode = True
    if "imageio" not in sys.modules:
        sys.modules["imageio"] = types.ModuleType("imageio")
    sys.path.insert(0, os.path.join(ref_root, "src"))
    import model as ref_model   # noqa
    import utils as ref_utils   # noqa
    sys.path.pop(0)
    return ref_model, ref_utils


def grad_digest(g, key_rng, n_pick=512):
    """Compact, strong fingerprint of a gradient tensor: sum, sum of squares,
    projection on a seeded random vector and a seeded subsample."""
    g = g.detach().double().reshape(-1).numpy()
    proj_vec = key_rng.standard_normal(g.size)
    idx = key_rng.choice(g.size, size=min(n_pick, g.size), replace=False)
    return dict(sum=g.sum(), sumsq=(g * g).sum(), proj=(g * proj_vec).sum(),
                idx=idx.astype(np.int64), vals=g[idx].astype(np.float32))


def run_case(ref_model, ref_utils, name, H, W, N, near, far, seed, chunk=2048,
             sigma_shift=0.0, radius=1.3, az=30.0, el=20.0, focal=131.25, n_obj=2,
             obj_idx=1, full_grads=False, store_samples=True):
    net = dict(shape_blocks=3, texture_blocks=1, W=256, num_xyz_freq=10,
               num_dir_freq=4, latent_dim=256)
    npp = make_params(seed, sigma_bias_shift=sigma_shift)
    model = ref_model.CodeNeRF(**net)
    model.load_state_dict({k: torch.tensor(v) for k, v in npp.items()})
    s_tab, t_tab = make_codes(seed, n_obj)
    shape_codes = torch.nn.Embedding(n_obj, 256)
    texture_codes = torch.nn.Embedding(n_obj, 256)
    shape_codes.weight = torch.nn.Parameter(torch.tensor(s_tab))
    texture_codes.weight = torch.nn.Parameter(torch.tensor(t_tab))

    g = torch.Generator().manual_seed(seed)
    jitter = torch.rand(N, generator=g)
    gt = torch.rand(H * W, 3, generator=g)
    c2w = torch.tensor(look_at_pose(radius, az, el))
    focal_t = torch.tensor([focal], dtype=torch.float64)    # as default_collate makes it

    rays_o, viewdir = ref_utils.get_rays(H, W, focal_t, c2w)
    # sample_from_rays draws its jitter with torch.rand(N) from the global
    # generator (src/utils.py:29); hand it our recorded draw instead
    orig_rand = torch.rand
    torch.rand = lambda *a, **k: jitter.clone()
    try:
        xyz, vd_rep, z_vals = ref_utils.sample_from_rays(rays_o, viewdir, near, far, N)
    finally:
        torch.rand = orig_rand

    out = dict(H=H, W=W, N=N, near=near, far=far, focal=focal, c2w=c2w.numpy(),
               jitter=jitter.numpy(), gt=gt.numpy(), seed=seed, chunk=chunk,
               sigma_shift=sigma_shift, obj_idx=obj_idx, n_obj=n_obj,
               rays_o=rays_o.numpy(), viewdir=viewdir.numpy(), z_vals=z_vals.numpy(),
               shape_table=s_tab, texture_table=t_tab)

    # --- forward of the whole image (no grad) + per-sample outputs ----------
    oi = torch.tensor([obj_idx])
    with torch.no_grad():
        sig, rgbs = model(xyz, vd_rep, shape_codes(oi), texture_codes(oi))
        rgb, depth = ref_utils.volume_rendering(sig, rgbs, z_vals)
    out.update(rgb=rgb.numpy(), depth=depth.numpy())
    if store_samples:
        out.update(sigmas=sig.numpy(), rgbs=rgbs.numpy())

    # --- one training image step, replaying src/trainer.py:64-85 ------------
    hp_lr = (1e-4, 1e-3)
    opts = torch.optim.AdamW([
        {"params": model.parameters(), "lr": hp_lr[0]},
        {"params": shape_codes.parameters(), "lr": hp_lr[1]},
        {"params": texture_codes.parameters(), "lr": hp_lr[1]},
    ])
    opts.zero_grad()
    loss_per_img, gen = [], []
    for i in range(0, xyz.shape[0], chunk):
        shape_code, texture_code = shape_codes(oi), texture_codes(oi)
        sigmas, rgbs_c = model(xyz[i:i + chunk], vd_rep[i:i + chunk], shape_code, texture_code)
        rgb_rays, _ = ref_utils.volume_rendering(sigmas, rgbs_c, z_vals)
        loss_l2 = torch.mean((rgb_rays - gt[i:i + chunk].type_as(rgb_rays)) ** 2)
        if i == 0:
            reg_loss = torch.norm(shape_code, dim=-1) + torch.norm(texture_code, dim=-1)
            loss = loss_l2 + 1e-4 * torch.mean(reg_loss)
        else:
            loss = loss_l2
        loss.backward()
        loss_per_img.append(loss_l2.item())
        gen.append(rgb_rays.detach())
    out["chunk_losses"] = np.array(loss_per_img)
    out["reg_loss"] = float(reg_loss.item())

    key_rng = np.random.Generator(np.random.PCG64(1234))
    names = [k for k, _ in model.named_parameters()]
    for k, prm in model.named_parameters():
        d = grad_digest(prm.grad, key_rng)
        for kk, vv in d.items():
            out[f"grad/{k}/{kk}"] = vv
        if full_grads:
            out[f"gradfull/{k}"] = prm.grad.numpy()
    out["grad/shape_table"] = shape_codes.weight.grad.numpy()
    out["grad/texture_table"] = texture_codes.weight.grad.numpy()

    opts.step()
    key_rng = np.random.Generator(np.random.PCG64(4321))
    for k, prm in model.named_parameters():
        d = grad_digest(prm.data, key_rng)
        out[f"adamw/{k}/idx"] = d["idx"]
        out[f"adamw/{k}/vals"] = d["vals"]
        out[f"adamw/{k}/sum"] = d["sum"]
    out["adamw/shape_table"] = shape_codes.weight.data.numpy()
    out["adamw/texture_table"] = texture_codes.weight.data.numpy()
    out["param_names"] = np.array(names)
    path = os.path.join(GOLD, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}  ({os.path.getsize(path) / 1024:.0f} KiB)  "
          f"psnr={-10 * math.log10(np.mean(loss_per_img)):.3f}")


def run_pe_and_render(ref_model, ref_utils):
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(257, 3, generator=g) * 4 - 2)
    d = torch.nn.functional.normalize(torch.randn(64, 3, generator=g), dim=-1)
    pe10 = ref_model.PE(x, 10)
    pe4 = ref_model.PE(d, 4)
    # volume rendering on random fields, incl. very dense / empty samples
    R, N = 96, 48
    sig = torch.rand(R, N, 1, generator=g) * 5
    sig[:16] *= 40.0           # dense rays: alpha -> 1, transmittance -> ~1e-10 products
    sig[16:24] = 0.0           # empty rays: background only
    rgbs = torch.rand(R, N, 3, generator=g) * 1.4 - 0.2     # unbounded rgb head
    z = torch.sort(torch.rand(N, generator=g) * 1.0 + 0.8).values
    sig.requires_grad_(True)
    rgbs.requires_grad_(True)
    rgb, depth = ref_utils.volume_rendering(sig, rgbs, z)
    drgb = torch.randn(R, 3, generator=g)
    ddepth = torch.randn(R, generator=g)
    (rgb * drgb).sum().add((depth * ddepth).sum()).backward()
    path = os.path.join(GOLD, "pe_render.npz")
    np.savez_compressed(path, x=x.numpy(), d=d.numpy(), pe10=pe10.numpy(), pe4=pe4.numpy(),
                        sig=sig.detach().numpy(), rgbs=rgbs.detach().numpy(), z=z.numpy(),
                        rgb=rgb.detach().numpy(), depth=depth.detach().numpy(),
                        drgb=drgb.numpy(), ddepth=ddepth.numpy(),
                        dsig=sig.grad.numpy(), drgbs=rgbs.grad.numpy())
    print("wrote", path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    os.makedirs(GOLD, exist_ok=True)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref_model, ref_utils = import_reference(args.ref)
    run_pe_and_render(ref_model, ref_utils)
    # C1 of SURVEY.md 8(d): 32x32 crop, N=32, srncar near/far
    run_case(ref_model, ref_utils, "c1_32x32_n32", 32, 32, 32, 0.8, 1.8, seed=0)
    # dense: sigma bias +25 -> softplus threshold branch, alpha -> 1, 1e-10 term
    run_case(ref_model, ref_utils, "dense_16x16_n32", 16, 16, 32, 0.8, 1.8, seed=1, sigma_shift=25.0)
    # one wave per ray (N=64) and the JSON default N=96, and N=128
    run_case(ref_model, ref_utils, "n64_16x16", 16, 16, 64, 0.8, 1.8, seed=2)
    run_case(ref_model, ref_utils, "n96_16x16_chairs", 16, 16, 96, 1.25, 2.75, seed=3, radius=2.0, az=-70.0, el=35.0)
    run_case(ref_model, ref_utils, "n128_8x8", 8, 8, 128, 0.8, 1.8, seed=4)
    # multi-chunk gradient semantics: 64x64 = 4096 rays = two 2048-ray chunks;
    # a ragged last chunk with chunk=1500
    run_case(ref_model, ref_utils, "chunks_64x64_n16", 64, 64, 16, 0.8, 1.8, seed=5, store_samples=False)
    run_case(ref_model, ref_utils, "ragged_48x48_n16", 48, 48, 16, 0.8, 1.8, seed=6, chunk=1500,
             store_samples=False)


if __name__ == "__main__":
    main()
