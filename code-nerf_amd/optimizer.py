"""Test-time code optimisation and evaluation on the HIP path
(reference: src/optimizer.py; BASELINE config 4).

Same API (``Optimizer(saved_dir, gpu, instance_ids, splits, jsonfile,
batch_size, num_opts).optimize_objs(instance_ids, lr, lr_half_interval,
save_img)``) and loop semantics:

  * codes start at the mean of the trained code tables (:232-233) and only
    the two codes are optimised (AdamW, lr halved every ``lr_half_interval``
    steps by re-creating the optimiser, :104-105,207-218);
  * one step = zero_grad, then every target view's image (chunked MSE + the
    code regulariser on each view's chunk 0) accumulates gradients, then
    one AdamW step (:66-98);
  * evaluation: every view that is not a target, forward only, PSNR from the
    mean of the chunk MSEs and SSIM (:108-130); with torch.distributed the
    views are split across ranks (dp.shard) and the metrics gathered
    (dp.gather_by_key), the z jitter of every view drawn first in view order
    so a split changes no draw;
  * ``codes.pth`` with the reference's keys (:138-145).
The model weights are fixed, so the weight-gradient pass is skipped (only the
dX chain and the code gradients run).  SSIM is ``metrics.ssim_legacy`` -- a
restatement of skimage's ``structural_similarity(multichannel=True)`` as the
reference calls it (skimage is not installed: parity unpinned).
"""
import json
import os
import time

import numpy as np
import torch

from . import dp
from .data import SRN, collate_one
from .metrics import ssim_legacy
from .model import CodeNeRF
from .optim import FusedAdamW
from .render import ImageStep
from .trainer import load_hpams
from .utils import get_rays, image_float_to_uint8


class Optimizer:
    def __init__(self, saved_dir, gpu=0, instance_ids=(), splits="test", jsonfile="srncar.json",
                 batch_size=2048, num_opts=200, hpams=None, exp_root="exps", dist=None):
        self.hpams = hpams if hpams is not None else load_hpams(jsonfile)
        self.device = torch.device("cuda", int(gpu))
        torch.cuda.set_device(self.device)
        self.exp_root = exp_root
        self.dist = dist
        self.world, self.rank = dp.world_rank(dist)
        self.make_model()
        self.load_model_codes(saved_dir)
        self.make_dataloader(splits, len(instance_ids))
        self.B = int(batch_size)
        self.num_opts = int(num_opts)
        self.splits = splits
        self.nviews = str(len(instance_ids))
        self.psnr_eval, self.psnr_opt, self.ssim_eval = {}, {}, {}
        self.step_impl = ImageStep(self.model, chunk=self.B, reg_coef=self.hpams["loss_reg_coef"])

    def _z_vals(self):
        near, far, N = self.hpams["near"], self.hpams["far"], self.hpams["N_samples"]
        half = (far - near) / (2 * N)
        z = torch.linspace(near + half, far - half, N)
        z += torch.rand(N) * (far - near) / (2 * N)
        return z.to(self.device)

    def optimize_objs(self, instance_ids, lr=1e-2, lr_half_interval=50, save_img=True):
        if self.rank == 0:
            with open(os.path.join(self.save_dir, "opt_hpams.json"), "w") as f:
                json.dump({"instance_ids": list(map(int, instance_ids)), "lr": lr,
                           "lr_half_interval": lr_half_interval, "": self.splits}, f, indent=2)
        self.lr, self.lr_half_interval = lr, lr_half_interval
        instance_ids = [int(i) for i in instance_ids]
        n = len(self.dataset)
        self.optimized_shapecodes = torch.zeros(n, self.mean_shape.shape[1])
        self.optimized_texturecodes = torch.zeros(n, self.mean_texture.shape[1])
        for num_obj in range(n):
            focal, H, W, imgs, poses, obj_idx = collate_one(self.dataset[num_obj])
            H, W = int(H), int(W)
            self.nopts = 0
            shapecode = self.mean_shape.to(self.device).clone().detach().requires_grad_()
            texturecode = self.mean_texture.to(self.device).clone().detach().requires_grad_()
            self.set_optimizers(shapecode, texturecode)
            while self.nopts < self.num_opts:
                shapecode.grad = torch.zeros_like(shapecode)
                texturecode.grad = torch.zeros_like(texturecode)
                t1 = time.time()
                gens, gts = [], []
                for num, iid in enumerate(instance_ids):
                    tgt_img = imgs[0, iid].reshape(-1, 3).to(self.device)
                    rays_o, viewdir = get_rays(H, W, focal, poses[0, iid])
                    losses, rgb, reg = self.step_impl.forward_backward(
                        rays_o, viewdir, self._z_vals(), tgt_img, shapecode, texturecode, 0, weight_grads=False)
                    gens.append(rgb.reshape(H, W, 3))
                    gts.append(tgt_img.reshape(H, W, 3))
                self.opts.step()
                self.log_opt_psnr(float(losses.mean()), time.time() - t1, num_obj)
                if save_img and self.rank == 0:
                    self.save_img(gens, gts, self.ids[num_obj], self.nopts)
                self.nopts += 1
                if self.nopts % lr_half_interval == 0:
                    self.set_optimizers(shapecode, texturecode)
            with torch.no_grad():
                # evaluation views (src/optimizer.py:108-130), split across
                # ranks when data parallel; the z jitter of every view is drawn
                # first, in view order, so the split does not change any draw
                views = [num for num in range(imgs.shape[1]) if num not in instance_ids]
                zs = {num: self._z_vals() for num in views}
                local = {}
                for num in dp.shard(views, self.dist):
                    tgt_img = imgs[0, num].reshape(-1, 3).to(self.device)
                    rays_o, viewdir = get_rays(H, W, focal, poses[0, num])
                    rgb, _ = self.step_impl.render(rays_o, viewdir, zs[num], shapecode, texturecode)
                    se = ((rgb - tgt_img) ** 2).sum(-1)
                    chunk_mse = [float(se[i:i + self.B].mean()) / 3 for i in range(0, H * W, self.B)]
                    local[num] = (float(-10 * np.log(float(np.mean(chunk_mse))) / np.log(10)),
                                  ssim_legacy(rgb.reshape(H, W, 3).cpu().numpy(),
                                              tgt_img.reshape(H, W, 3).cpu().numpy()))
                    if save_img:
                        self.save_img([rgb.reshape(H, W, 3)], [tgt_img.reshape(H, W, 3)], self.ids[num_obj], num,
                                      opt=False)
                for num, (psnr, ssim) in dp.gather_by_key(local, self.dist).items():
                    self.psnr_eval.setdefault(num_obj, []).append(psnr)
                    self.ssim_eval.setdefault(num_obj, []).append(ssim)
            self.optimized_shapecodes[num_obj] = shapecode.detach().cpu()
            self.optimized_texturecodes[num_obj] = texturecode.detach().cpu()
            self.save_opts(num_obj)

    def set_optimizers(self, shapecode, texturecode):
        lr = self.lr * 2 ** (-(self.nopts // self.lr_half_interval))
        self.opts = FusedAdamW([{"params": [shapecode], "lr": lr}, {"params": [texturecode], "lr": lr}])

    def log_opt_psnr(self, mse, time_spent, num_obj):
        self.psnr_opt.setdefault(num_obj, []).append(float(-10 * np.log(mse) / np.log(10)))

    def log_eval_psnr(self, mse, num_obj):
        self.psnr_eval.setdefault(num_obj, []).append(float(-10 * np.log(mse) / np.log(10)))

    def save_opts(self, num_obj):
        if self.rank != 0:
            return
        torch.save({"ids": [str(i) for i in self.ids], "num_obj": num_obj,
                    "optimized_shapecodes": self.optimized_shapecodes,
                    "optimized_texturecodes": self.optimized_texturecodes,
                    "psnr_eval": self.psnr_eval, "ssim_eval": self.ssim_eval},
                   os.path.join(self.save_dir, "codes.pth"))

    def save_img(self, generated_imgs, gt_imgs, obj_id, instance_num, opt=True):
        from PIL import Image
        H, W = gt_imgs[0].shape[:2]
        nv = len(generated_imgs)
        ret = torch.zeros(nv * H, 2 * W, 3)
        ret[:, :W] = torch.cat([g.detach().cpu() for g in generated_imgs]).reshape(-1, W, 3)
        ret[:, W:] = torch.cat([g.detach().cpu() for g in gt_imgs]).reshape(-1, W, 3)
        d = os.path.join(self.save_dir, str(obj_id))
        os.makedirs(d, exist_ok=True)
        name = f"opt{self.nviews}_{instance_num}.png" if opt else f"{instance_num}_{self.nviews}.png"
        Image.fromarray(image_float_to_uint8(ret.numpy())).save(os.path.join(d, name))

    def make_model(self):
        prec = self.hpams.get("precision", "fp32")
        self.model = CodeNeRF(**self.hpams["net_hyperparams"], precision=prec).to(self.device)

    def load_model_codes(self, saved_dir):
        saved = torch.load(os.path.join(self.exp_root, saved_dir, "models.pth"), map_location="cpu",
                           weights_only=True)
        self.make_save_img_dir(os.path.join(self.exp_root, saved_dir, "test"))
        self.model.load_state_dict(saved["model_params"])
        self.model = self.model.to(self.device)
        self.mean_shape = torch.mean(saved["shape_code_params"]["weight"], dim=0).reshape(1, -1)
        self.mean_texture = torch.mean(saved["texture_code_params"]["weight"], dim=0).reshape(1, -1)

    def make_save_img_dir(self, save_dir):
        # rank 0 picks the first free "test", "test_2", ... and tells the others
        tmp = None
        if self.rank == 0:
            tmp, num = save_dir, 2
            while os.path.isdir(tmp):
                tmp = save_dir + "_" + str(num)
                num += 1
            os.makedirs(tmp)
        if self.world > 1:
            box = [tmp]
            self.dist.broadcast_object_list(box, src=0)
            tmp = box[0]
        self.save_dir = tmp

    def make_dataloader(self, splits, num_instances_per_obj, crop_img=False):
        d = self.hpams["data"]
        obj = d["cat"].split("_")[1]
        self.dataset = SRN(cat=d["cat"], splits=obj + "_" + splits, data_dir=d["data_dir"],
                           num_instances_per_obj=num_instances_per_obj, crop_img=crop_img,
                           n_test_views=int(d.get("n_test_views", 250)))
        self.ids = self.dataset.ids
