"""One optimisation step of CodeNeRF training on one device (or one rank).

Mirrors the per-object body of the reference loop (src/trainer.py:58-85):
rays from the pose, stratified z, the fused image forward/backward
(render.ImageStep; with n_fine > 0 the coarse + fine step, an extension the
reference lacks), then AdamW over the model and both code tables
(src/trainer.py:114-120).  Gradients live in one flat fp32 buffer (every
``.grad`` is a view into it), so zeroing is one memset and the data-parallel
exchange is one RCCL all-reduce of 2.9 MB + the code tables per step.
"""
import torch

from . import engine as _eng
from .dp import GradBucket
from .optim import FusedAdamW
from .render import ImageStep


class TrainCore:
    def __init__(self, model, shape_codes, texture_codes, near, far, n_coarse, n_fine=0, chunk=2048,
                 reg_coef=1e-4, lr=(1e-4, 1e-3), timers=None, dist=None):
        self.model = model
        self.shape_codes = shape_codes
        self.texture_codes = texture_codes
        self.near, self.far = float(near), float(far)
        self.n_coarse = int(n_coarse)
        self.n_fine = int(n_fine)
        self.dist = dist
        self.step_impl = ImageStep(model, chunk=chunk, reg_coef=reg_coef, timers=timers)
        self.bucket = GradBucket(model.param_list() + [shape_codes, texture_codes])
        self.flat_grad = self.bucket.flat
        self.opt = FusedAdamW([{"params": model.param_list(), "lr": lr[0]},
                               {"params": [shape_codes], "lr": lr[1]},
                               {"params": [texture_codes], "lr": lr[1]}])

    def stratified_z(self, device):
        n = self.n_coarse
        half = (self.far - self.near) / (2 * n)
        z = torch.linspace(self.near + half, self.far - half, n, device=device)
        return z + torch.rand(n, device=device) * (self.far - self.near) / (2 * n)

    def train_step(self, H, W, focal, c2w, gt, obj, ray_parts=1):
        """ray_parts > 1 renders the image as that many contiguous ray ranges
        (each a multiple of the loss chunk, so the chunk-mean semantics are
        unchanged; the regulariser is counted once, on the first part) whose
        gradients accumulate before the one AdamW step: bounds the activation
        workspace for large images (C5: 256^2 x 256 samples in fp32)."""
        dev = c2w.device
        ro, vd = _eng.get_rays_dev(H, W, focal, True, c2w)
        z = self.stratified_z(dev)
        self.bucket.zero()
        R = H * W
        if R % ray_parts or (R // ray_parts) % self.step_impl.chunk:
            raise ValueError("ray_parts must split the image into whole loss chunks")
        P = R // ray_parts
        rand_f = torch.rand(R, self.n_fine, device=dev) if self.n_fine else None
        losses, rgbs = [], []
        for k in range(ray_parts):
            sl = slice(k * P, (k + 1) * P)
            if self.n_fine:
                loss_c, loss_f, rgb, _ = self.step_impl.forward_backward_fine(
                    ro[sl], vd[sl], z, rand_f[sl], gt[sl], self.shape_codes, self.texture_codes, obj, reg=k == 0)
                losses.append((loss_c, loss_f))
            else:
                loss, rgb, _ = self.step_impl.forward_backward(ro[sl], vd[sl], z, gt[sl], self.shape_codes,
                                                              self.texture_codes, obj, reg=k == 0)
                losses.append(loss)
            rgbs.append(rgb)
        self.bucket.all_reduce(self.dist)
        self.opt.step()
        if ray_parts == 1:
            return losses[0], rgbs[0]
        if self.n_fine:
            return (torch.cat([l[0] for l in losses]), torch.cat([l[1] for l in losses])), torch.cat(rgbs)
        return torch.cat(losses), torch.cat(rgbs)
