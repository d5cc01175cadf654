"""Seeded parameters in the reference's state_dict order (test infrastructure).

The reference registers its sub-modules in this order (src/model.py:20-34):
encoding_xyz, then per shape block ``shape_latent_layer_j`` / ``shape_layer_j``,
encoding_shape, sigma, encoding_viewdir, per texture block
``texture_latent_layer_j`` / ``texture_layer_j``, rgb.  nn.Linear stores its
weight as (out, in).  Values come from numpy's PCG64 so the same tensors are
reproduced on any machine (torch's CPU RNG is not relied upon); the
distribution is nn.Linear's default U(-1/sqrt(fan_in), 1/sqrt(fan_in)).
"""
from collections import OrderedDict

import numpy as np

DEFAULT_NET = dict(shape_blocks=3, texture_blocks=1, W=256,
                   num_xyz_freq=10, num_dir_freq=4, latent_dim=256)


def param_specs(shape_blocks=3, texture_blocks=1, W=256, num_xyz_freq=10,
                num_dir_freq=4, latent_dim=256):
    """[(name, shape)] in reference registration order."""
    d_xyz = 3 + 6 * num_xyz_freq
    d_dir = 3 + 6 * num_dir_freq
    specs = []

    def lin(prefix, n_in, n_out):
        specs.append((prefix + ".weight", (n_out, n_in)))
        specs.append((prefix + ".bias", (n_out,)))

    lin("encoding_xyz.0", d_xyz, W)
    for j in range(1, shape_blocks + 1):
        lin(f"shape_latent_layer_{j}.0", latent_dim, W)
        lin(f"shape_layer_{j}.0", W, W)
    lin("encoding_shape", W, W)
    lin("sigma.0", W, 1)
    lin("encoding_viewdir.0", W + d_dir, W)
    for j in range(1, texture_blocks + 1):
        lin(f"texture_latent_layer_{j}.0", latent_dim, W)
        lin(f"texture_layer_{j}.0", W, W)
    lin("rgb.0", W, W // 2)
    lin("rgb.2", W // 2, 3)
    return specs


def make_params(seed=0, sigma_bias_shift=0.0, **net):
    """OrderedDict name -> float32 ndarray, deterministic in ``seed``."""
    cfg = dict(DEFAULT_NET)
    cfg.update(net)
    rng = np.random.Generator(np.random.PCG64(seed))
    out = OrderedDict()
    for name, shape in param_specs(**cfg):
        fan_in = shape[1] if len(shape) == 2 else None
        if fan_in is None:  # bias: fan_in of the matching weight
            fan_in = out[name[:-len("bias")] + "weight"].shape[1]
        bound = 1.0 / np.sqrt(fan_in)
        out[name] = rng.uniform(-bound, bound, size=shape).astype(np.float32)
    if sigma_bias_shift:
        out["sigma.0.bias"] = (out["sigma.0.bias"] + np.float32(sigma_bias_shift)).astype(np.float32)
    return out


def make_codes(seed, n_obj, latent_dim=256):
    """Code tables like src/trainer.py:138-139 (randn / sqrt(dim/2)), numpy RNG."""
    rng = np.random.Generator(np.random.PCG64(seed + 7919))
    s = rng.standard_normal((n_obj, latent_dim)) / np.sqrt(latent_dim / 2)
    t = rng.standard_normal((n_obj, latent_dim)) / np.sqrt(latent_dim / 2)
    return s.astype(np.float32), t.astype(np.float32)


def look_at_pose(radius, azimuth_deg, elevation_deg):
    """OpenGL-convention camera-to-world (x right, y up, camera looks down -z)
    on a sphere around the origin, as SRN poses are after the diag(1,-1,-1,1)
    flip of src/data.py:13,16-17."""
    az, el = np.deg2rad(azimuth_deg), np.deg2rad(elevation_deg)
    eye = radius * np.array([np.cos(el) * np.sin(az), np.sin(el), np.cos(el) * np.cos(az)])
    fwd = -eye / np.linalg.norm(eye)            # viewing direction
    up = np.array([0.0, 1.0, 0.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    true_up = np.cross(right, fwd)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = right, true_up, -fwd, eye
    return c2w.astype(np.float32)
