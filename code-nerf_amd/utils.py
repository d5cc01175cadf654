"""Reference-API geometry / rendering helpers on the HIP device.

Same names, arguments and return shapes as the reference's src/utils.py so the
loops read the same:

  get_rays(H, W, focal, c2w) -> (rays_o, viewdirs)           src/utils.py:10-19
  sample_from_rays(ro, vd, near, far, N_samples, z_fixed)    src/utils.py:21-32
  volume_rendering(sigmas, rgbs, z_vals, white_bg=True)      src/utils.py:34-47
  image_float_to_uint8, str2bool                              src/utils.py:49-71

Inputs may live on the host (the reference builds rays on the CPU); they are
moved to the current HIP device and every computation runs in the HIP
library.  The stratified jitter is still drawn with ``torch.rand`` from the
global CPU generator, exactly as the reference does, so seeded runs draw the
same z values.
"""
import argparse

import numpy as np
import torch

from . import engine as _eng


def _device():
    return torch.device("cuda", torch.cuda.current_device())


def get_rays(H, W, focal, c2w):
    """Pinhole rays, OpenGL camera convention, principal point (W/2, H/2),
    no half-pixel offset.  ``focal`` as a float64 tensor (what default_collate
    yields) makes the camera directions float64 before the cast, like the
    reference's type promotion."""
    dev = c2w.device if c2w.is_cuda else _device()
    if isinstance(focal, torch.Tensor):
        f64 = focal.dtype == torch.float64
        fval = float(focal.reshape(-1)[0])
    else:
        f64, fval = False, float(focal)
    m = c2w.reshape(-1, 4, 4)[0, :4, :4].to(dev, torch.float32).contiguous()
    return _eng.get_rays_dev(int(H), int(W), fval, f64, m)


def stratified_z(near, far, n_samples, z_fixed=False):
    """z values of src/utils.py:24-29 (one vector shared by all rays)."""
    if z_fixed:
        return torch.linspace(near, far, n_samples)
    half = (far - near) / (2 * n_samples)
    z = torch.linspace(near + half, far - half, n_samples)
    z += torch.rand(n_samples) * (far - near) / (2 * n_samples)
    return z


def sample_from_rays(ro, vd, near, far, N_samples, z_fixed=False):
    """-> xyz (R,N,3), viewdir (R,N,3), z_vals (N,), all on the HIP device."""
    dev = ro.device if ro.is_cuda else _device()
    z = stratified_z(near, far, N_samples, z_fixed).to(dev, torch.float32)
    ro = ro.to(dev, torch.float32).contiguous()
    vd = vd.to(dev, torch.float32).contiguous()
    xyz, vrep = _eng.sample_points(ro, vd, z, ro.shape[0], N_samples)
    return xyz, vrep, z


class _VolumeRendering(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sigmas, rgbs, z_vals, white_bg):
        R, N = rgbs.shape[0], rgbs.shape[1]
        s = sigmas.contiguous().reshape(R * N).to(torch.float32)
        c = rgbs.contiguous().reshape(R * N, 3).to(torch.float32)
        z = z_vals.contiguous().to(torch.float32)
        if z.numel() not in (N, R * N):
            raise ValueError("z_vals must be (N,) or (R, N)")
        out_rgb, depth = _eng.composite_fwd(s, c, z, R, N, white_bg)
        ctx.save_for_backward(s, c, z)
        ctx.dims = (R, N, white_bg)
        return out_rgb, depth

    @staticmethod
    def backward(ctx, g_rgb, g_depth):
        s, c, z = ctx.saved_tensors
        R, N, white_bg = ctx.dims
        if g_rgb is None:
            g_rgb = torch.zeros(R, 3, device=s.device)
        dsig, drgb = _eng.composite_bwd(s, c, z, R, N, g_rgb.contiguous().to(torch.float32),
                                        None if g_depth is None else g_depth.contiguous().to(torch.float32),
                                        white_bg)
        return dsig.reshape(R, N, 1), drgb.reshape(R, N, 3), None, None


def volume_rendering(sigmas, rgbs, z_vals, white_bg=True):
    """Alpha compositing along each ray -> (rgb (R,3), depth (R,))."""
    if not sigmas.is_cuda:
        raise RuntimeError("volume_rendering (MI355X) expects HIP tensors")
    return _VolumeRendering.apply(sigmas, rgbs, z_vals.to(sigmas.device), bool(white_bg))


def image_float_to_uint8(img):
    """Min-max normalise to uint8 (src/utils.py:49-60), host-side image I/O."""
    vmin, vmax = np.min(img), np.max(img)
    if vmax - vmin < 1e-10:
        vmax += 1e-10
    return ((img - vmin) / (vmax - vmin) * 255.0).astype(np.uint8)


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true"):
        return True
    if v.lower() in ("no", "false"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")
