"""CodeNeRF training loop on the HIP path (reference: src/trainer.py).

Same constructor / ``training(iters_crop, iters_all, num_instances_per_obj)``
API and the same loop semantics, kept deliberately:

  * an epoch visits every object once (DataLoader order, batch 1); the
    optimiser (AdamW over model + both code tables) is RE-CREATED at the start
    of every epoch with the step-halved learning rates (src/trainer.py:52,
    122-133), so its moments restart each epoch;
  * per object, ``zero_grad`` runs inside the per-image loop (:62-64), so
    only the last of the ``num_instances_per_obj`` images drives the step;
  * per image: rays, stratified z from the global CPU generator, chunks of B
    rays with chunk-mean MSE, the code regulariser on chunk 0 (:65-84) -- one
    fused ``ImageStep`` call here;
  * checkpoints: ``models.pth`` (+ ``<iter>.pth`` every ``check_points``)
    with the reference's keys (:166-170).
Logging goes to ``<save_dir>/runs/log.jsonl`` (tensorboard is not
installed); images every ``check_iter`` iterations to ``<save_dir>/img``.

Extensions (JSON keys the reference ignores): ``N_importance`` (fine
samples per ray, the BASELINE "+fine"), ``precision`` ("fp32" | "bf16").
With torch.distributed initialised, rank r trains object
``dp.object_for(step, r, world, n_obj)`` and gradients are all-reduced.
"""
import json
import math
import os
import time

import numpy as np
import torch

from . import dp
from .data import SRN, collate_one
from .model import CodeNeRF
from .optim import FusedAdamW
from .render import ImageStep
from .utils import get_rays, image_float_to_uint8


def load_hpams(jsonfile, search=("configs", "jsonfiles")):
    path = jsonfile
    if not os.path.exists(path):
        for d in search:
            cand = os.path.join(d, jsonfile)
            if os.path.exists(cand):
                path = cand
                break
    with open(path) as f:
        return json.load(f)


class Trainer:
    def __init__(self, save_dir, gpu=0, jsonfile="srncar.json", batch_size=2048, check_iter=10000,
                 hpams=None, exp_root="exps", dist=None):
        self.hpams = hpams if hpams is not None else load_hpams(jsonfile)
        self.device = torch.device("cuda", int(gpu))
        torch.cuda.set_device(self.device)
        self.dist = dist
        self.rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
        self.make_model()
        self.make_dataloader(num_instances_per_obj=1, crop_img=False)
        self.make_codes()
        self.B = int(batch_size)
        self.make_savedir(save_dir, exp_root)
        self.niter, self.nepoch = 0, 0
        self.check_iter = int(check_iter)
        self.step_impl = ImageStep(self.model, chunk=self.B, reg_coef=self.hpams["loss_reg_coef"])
        self.exchange = dp.GradExchange(self.model.param_list(), [self.shape_codes.weight, self.texture_codes.weight],
                                        dist)
        self.step_impl.grad_listeners.append(self.exchange.mark_dirty)     # every .grad write re-arms zero()
        self.n_fine = int(self.hpams.get("N_importance", 0))
        self.psnr_log = []

    # ---------------------------------------------------------------- loop
    def training(self, iters_crop, iters_all, num_instances_per_obj=1):
        if iters_crop > iters_all:
            raise ValueError("iters_crop must not exceed iters_all")
        while self.niter < iters_all:
            if self.niter < iters_crop:
                self.training_single_epoch(num_instances_per_obj, iters_crop, crop_img=True)
            else:
                self.training_single_epoch(num_instances_per_obj, iters_all, crop_img=False)
            self.save_models()
            self.nepoch += 1

    def _z_vals(self, N):
        near, far = self.hpams["near"], self.hpams["far"]
        half = (far - near) / (2 * N)
        z = torch.linspace(near + half, far - half, N)
        z += torch.rand(N) * (far - near) / (2 * N)          # global CPU generator, src/utils.py:29
        return z.to(self.device)

    def training_single_epoch(self, num_instances_per_obj, num_iters, crop_img=True):
        self.make_dataloader(num_instances_per_obj, crop_img=crop_img)
        self.set_optimizers()
        n_obj = len(self.dataset)
        order = range(n_obj) if self.world == 1 else \
            [dp.object_for(s, self.rank, self.world, n_obj) for s in range((n_obj + self.world - 1) // self.world)]
        for idx in order:
            if self.niter >= num_iters:
                break
            focal, H, W, imgs, poses, instances, obj_idx = collate_one(self.dataset[idx])
            H, W, oi = int(H), int(W), int(obj_idx)
            t1 = time.time()
            for k in range(num_instances_per_obj):
                self.exchange.zero()                                # zero_grad inside the image loop
                rays_o, viewdir = get_rays(H, W, focal, poses[0, k])
                z = self._z_vals(self.hpams["N_samples"])
                gt = imgs[0, k].to(self.device).contiguous()
                if self.n_fine:
                    rnd = torch.rand(H * W, self.n_fine, device=self.device)
                    lc, lf, rgb, reg = self.step_impl.forward_backward_fine(
                        rays_o, viewdir, z, rnd, gt, self.shape_codes.weight, self.texture_codes.weight, oi)
                    loss_per_img = lf
                else:
                    loss_per_img, rgb, reg = self.step_impl.forward_backward(
                        rays_o, viewdir, z, gt, self.shape_codes.weight, self.texture_codes.weight, oi)
            self.exchange.exchange_rows([oi], 1)          # data parallel: the touched code rows,
            work = self.exchange.start_model()           # then the async model all-reduce
            self.opts.step(groups=[1, 2], zero_grad=True)  # the kernel leaves the gradients at 0:
            self.exchange.finish(work)
            self.opts.step(groups=[0], zero_grad=True)
            self.exchange.clean = True                     # the next zero_grad needs no launch
            mse = float(loss_per_img.mean())
            self.log_psnr_time(mse, time.time() - t1, oi, float(reg))
            if self.check_iter and self.niter % self.check_iter == 0:
                self.log_img(rgb.reshape(H, W, 3), imgs[0, -1].reshape(H, W, 3), oi)
            if self.niter % self.hpams["check_points"] == 0:
                self.save_models(self.niter)
            self.niter += 1

    # ---------------------------------------------------------------- pieces
    def get_learning_rate(self):
        model_lr, latent_lr = self.hpams["lr_schedule"][0], self.hpams["lr_schedule"][1]
        lr1 = model_lr["lr"] * 2 ** (-(self.niter // model_lr["interval"]))
        lr2 = latent_lr["lr"] * 2 ** (-(self.niter // latent_lr["interval"]))
        return lr1, lr2

    def set_optimizers(self):
        lr1, lr2 = self.get_learning_rate()
        self.opts = FusedAdamW([{"params": self.model.param_list(), "lr": lr1},
                                {"params": [self.shape_codes.weight], "lr": lr2},
                                {"params": [self.texture_codes.weight], "lr": lr2}])

    def make_model(self):
        prec = self.hpams.get("precision", "fp32")
        self.model = CodeNeRF(**self.hpams["net_hyperparams"], precision=prec).to(self.device)
        dp.broadcast_from(list(self.model.parameters()), self.dist)

    def make_codes(self):
        embdim = self.hpams["net_hyperparams"]["latent_dim"]
        d = len(self.dataset)
        self.shape_codes = torch.nn.Embedding(d, embdim)
        self.texture_codes = torch.nn.Embedding(d, embdim)
        self.shape_codes.weight = torch.nn.Parameter(torch.randn(d, embdim) / math.sqrt(embdim / 2))
        self.texture_codes.weight = torch.nn.Parameter(torch.randn(d, embdim) / math.sqrt(embdim / 2))
        self.shape_codes = self.shape_codes.to(self.device)
        self.texture_codes = self.texture_codes.to(self.device)
        dp.broadcast_from([self.shape_codes.weight, self.texture_codes.weight], self.dist)

    def make_dataloader(self, num_instances_per_obj, crop_img):
        d = self.hpams["data"]
        self.dataset = SRN(cat=d["cat"], splits=d["splits"], data_dir=d["data_dir"],
                           num_instances_per_obj=num_instances_per_obj, crop_img=crop_img,
                           n_train_views=int(d.get("n_train_views", 50)))

    def make_savedir(self, save_dir, exp_root):
        self.save_dir = os.path.join(exp_root, save_dir)
        os.makedirs(os.path.join(self.save_dir, "runs"), exist_ok=True)
        if self.rank == 0:
            with open(os.path.join(self.save_dir, "hpam.json"), "w") as f:
                json.dump(self.hpams, f, indent=2)

    def log_psnr_time(self, mse, time_spent, obj_idx, reg):
        psnr = -10 * np.log(mse) / np.log(10)
        self.psnr_log.append(psnr)
        if self.rank == 0:
            with open(os.path.join(self.save_dir, "runs", "log.jsonl"), "a") as f:
                f.write(json.dumps({"iter": self.niter, "obj": obj_idx, "psnr/train": psnr,
                                    "time/train": time_spent, "reg/train": reg}) + "\n")

    def log_img(self, generated_img, gtimg, obj_idx):
        if self.rank != 0:
            return
        from PIL import Image
        H, W = generated_img.shape[:2]
        ret = torch.zeros(H, 2 * W, 3)
        ret[:, :W] = generated_img.detach().cpu()
        ret[:, W:] = gtimg.detach().cpu()
        os.makedirs(os.path.join(self.save_dir, "img"), exist_ok=True)
        Image.fromarray(image_float_to_uint8(ret.numpy())).save(
            os.path.join(self.save_dir, "img", f"train_{self.niter}_{obj_idx}.png"))

    def save_models(self, iter=None):
        if self.rank != 0:
            return
        save_dict = {"model_params": self.model.state_dict(),
                     "shape_code_params": self.shape_codes.state_dict(),
                     "texture_code_params": self.texture_codes.state_dict(),
                     "niter": self.niter, "nepoch": self.nepoch}
        if iter is not None:
            torch.save(save_dict, os.path.join(self.save_dir, f"{iter}.pth"))
        torch.save(save_dict, os.path.join(self.save_dir, "models.pth"))
