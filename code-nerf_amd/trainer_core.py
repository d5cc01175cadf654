"""One optimisation step of CodeNeRF training on one device (or one rank).

Mirrors the per-object body of the reference loop (src/trainer.py:58-85):
rays from the pose, stratified z, the fused image forward/backward
(render.ImageStep; with n_fine > 0 the coarse + fine step, an extension the
reference lacks), then AdamW over the model and both code tables
(src/trainer.py:114-120).  Model gradients live in one flat fp32 buffer
(every ``.grad`` is a view into it); the data-parallel exchange is one async
RCCL all-reduce of that 2.9 MB bucket plus an all_gather of the touched
code-table rows (dp.GradExchange).
"""
import torch

from . import engine as _eng
from .dp import GradExchange
from .optim import FusedAdamW
from .render import ImageStep


class TrainCore:
    def __init__(self, model, shape_codes, texture_codes, near, far, n_coarse, n_fine=0, chunk=2048,
                 reg_coef=1e-4, lr=(1e-4, 1e-3), timers=None, dist=None, step_opts=None, zero_grad_in_adamw=True,
                 rows_per_step=1):
        self.model = model
        self.shape_codes = shape_codes
        self.texture_codes = texture_codes
        self.near, self.far = float(near), float(far)
        self.n_coarse = int(n_coarse)
        self.n_fine = int(n_fine)
        self.dist = dist
        self.step_impl = ImageStep(model, chunk=chunk, reg_coef=reg_coef, timers=timers, **(step_opts or {}))
        self.exchange = GradExchange(model.param_list(), [shape_codes, texture_codes], dist)
        # any write into .grad (a direct ImageStep call included) re-arms zero()
        self.step_impl.grad_listeners.append(self.exchange.mark_dirty)
        # code rows each rank may exchange per step: every rank pads its rows
        # to this SAME constant, so the all_gather sizes agree without a
        # count exchange (exchange_rows raises past it)
        self.rows_per_step = int(rows_per_step)
        self.bucket = self.exchange.bucket
        self.flat_grad = self.bucket.flat
        # the AdamW kernel leaves the gradients it consumed at 0, so the next
        # step's zero_grad costs no launch (False keeps .grad readable after
        # train_step, for tests)
        self.zero_grad_in_adamw = bool(zero_grad_in_adamw)
        self.opt = FusedAdamW([{"params": model.param_list(), "lr": lr[0]},
                               {"params": [shape_codes], "lr": lr[1]},
                               {"params": [texture_codes], "lr": lr[1]}])

    def stratified_z(self, device):
        """src/utils.py:24-29 on the host, as the reference draws it (global
        CPU generator): one (N,) vector, copied to the device (no kernel)."""
        n = self.n_coarse
        half = (self.far - self.near) / (2 * n)
        z = torch.linspace(self.near + half, self.far - half, n)
        z = z + torch.rand(n) * (self.far - self.near) / (2 * n)
        return z.pin_memory().to(device, non_blocking=True)

    def train_step(self, H, W, focal, c2w, gt, obj):
        """One object step: rays, stratified z, the image forward/backward
        (ImageStep splits images beyond the activation budget into ray parts
        of whole loss chunks: C5's 256^2 x 256 samples in fp32), the
        gradient exchange, AdamW.  -> (losses, rendered rgb); with n_fine the
        losses are (coarse, fine) chunk losses."""
        dev = c2w.device
        ro, vd = _eng.get_rays_dev(H, W, focal, True, c2w)
        z = self.stratified_z(dev)
        self.exchange.zero()           # no launch when the last AdamW step left the gradients at 0
        if self.n_fine:
            rand_f = torch.rand(H * W, self.n_fine, device=dev)
            loss_c, loss_f, rgb, _ = self.step_impl.forward_backward_fine(
                ro, vd, z, rand_f, gt, self.shape_codes, self.texture_codes, obj)
            losses = (loss_c, loss_f)
        else:
            losses, rgb, _ = self.step_impl.forward_backward(ro, vd, z, gt, self.shape_codes, self.texture_codes,
                                                             obj)
        self.step_grads([obj])
        return losses, rgb

    def step_grads(self, rows):
        """Exchange (data parallel) and apply the gradients: the touched code
        rows are all-gathered first (a few KB: issued behind the 2.86 MB
        model all-reduce on the same communicator it would wait for it), then
        the model bucket's all-reduce is issued asynchronously and the code
        tables take their AdamW step while it is in flight; then the model's
        AdamW step."""
        self.exchange.mark_dirty()     # a backward filled the gradients
        self.exchange.exchange_rows(rows, self.rows_per_step)
        work = self.exchange.start_model()
        zg = self.zero_grad_in_adamw
        self.opt.step(groups=[1, 2], zero_grad=zg)
        self.exchange.finish(work)
        self.opt.step(groups=[0], zero_grad=zg)
        if zg:
            self.exchange.clean = True
