"""Thin host wrapper of the C ABI: one ``Engine`` = one plan (network
configuration + precision) on one device.

It owns the packed weight blobs (repacked only when a parameter changed), the
device pointer tables, and hands torch tensors to the ``cn_*`` entry points
on torch's current stream.  All arithmetic happens in the HIP library.
"""
import ctypes
import os

import torch
from torch.autograd.graph import increment_version

from . import _lib
from ._lib import check, ptr

PRECISIONS = {"fp32": _lib.CN_FP32, "bf16": _lib.CN_BF16, "bf16x3": _lib.CN_BF16X3, "bf16x3f": _lib.CN_BF16X3F}
# Training-workspace budget per call (bytes): larger images are rendered in
# ray parts that fit it (render.ImageStep, model.CodeNeRF.forward).  At the
# srncar net one training sample holds ~8.2 KB (bf16) / ~16 KB (fp32) of
# activation planes, so 48 GiB is ~6.2 M / ~3.1 M samples per part.
ACT_BUDGET = int(os.environ.get("CODENERF_ACT_BUDGET", str(48 << 30)))


class Engine:
    def __init__(self, shape_blocks=3, texture_blocks=1, W=256, num_xyz_freq=10, num_dir_freq=4,
                 latent_dim=256, precision="fp32", device=None):
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(PRECISIONS)}")
        self.L = _lib.lib()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.precision = precision
        self.net = dict(shape_blocks=shape_blocks, texture_blocks=texture_blocks, W=W,
                        num_xyz_freq=num_xyz_freq, num_dir_freq=num_dir_freq, latent_dim=latent_dim)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.L.cn_plan_create(shape_blocks, texture_blocks, W, num_xyz_freq, num_dir_freq, latent_dim,
                                        PRECISIONS[precision], ctypes.byref(h)), "cn_plan_create")
        self._plan = h
        self.n_params = self.L.cn_plan_num_params(h)
        self.n_inject = self.L.cn_plan_num_inject(h)
        self.blob_floats = self.L.cn_blob_floats(h)
        self.pack_fwd = torch.empty(self.L.cn_packed_bytes(h, 0), dtype=torch.uint8, device=self.device)
        self.pack_bwd = torch.empty(self.L.cn_packed_bytes(h, 1), dtype=torch.uint8, device=self.device)
        self._packed_key = None
        self._param_tab = None
        self._tables = {}

    def __del__(self):
        try:
            if getattr(self, "_plan", None) is not None and self._plan.value:
                self.L.cn_plan_destroy(self._plan)
        except Exception:
            pass

    # ------------------------------------------------------------ helpers
    @property
    def stream(self):
        return _lib.stream_ptr(self.device)

    def pad(self, M):
        return self.L.cn_pad_samples(self._plan, M)

    def act_bytes(self, M):
        return self.L.cn_act_bytes(self._plan, M)

    def dw_ws_bytes(self, M):
        return self.L.cn_dw_ws_bytes(self._plan, M)

    def act_bytes_per_sample(self):
        return self.L.cn_act_bytes_per_sample(self._plan)

    def max_act_samples(self, budget=None):
        """Most training samples one workspace of ``budget`` bytes holds
        (a multiple of the 256-sample tile, at most CN_MAX_SAMPLES)."""
        b = ACT_BUDGET if budget is None else int(budget)
        n = (b // self.act_bytes_per_sample()) // 256 * 256
        return max(256, min(n, self.L.cn_max_samples() // 256 * 256))

    def table(self, tensors):
        """Device array of the tensors' data pointers (cached)."""
        key = tuple(t.data_ptr() for t in tensors)
        tab = self._tables.get(key)
        if tab is None:
            if len(self._tables) > 64:
                self._tables.clear()
            tab = torch.tensor(list(key), dtype=torch.int64, device=self.device)
            self._tables[key] = tab
        return tab

    def _check_params(self, params):
        if len(params) != self.n_params:
            raise ValueError(f"expected {self.n_params} parameter tensors, got {len(params)}")
        for p in params:
            if p.device != self.device or p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("parameters must be contiguous float32 tensors on the engine's device")

    # ------------------------------------------------------------ weights
    def ensure_packed(self, params, bwd=True):
        key = (tuple((p.data_ptr(), p._version) for p in params), bwd)
        if key == self._packed_key:
            return
        self._check_params(params)
        tab = self.table(params)
        check(self.L.cn_pack_weights(self._plan, ptr(tab), ptr(self.pack_fwd),
                                     ptr(self.pack_bwd) if bwd else None, self.stream), "cn_pack_weights")
        self._packed_key = key
        self._param_tab = tab       # the weights the packs came from (mlp_dw's fold reads them)

    def latent_fwd(self, params, shape_code, texture_code):
        blob = torch.empty(self.blob_floats, dtype=torch.float32, device=self.device)
        zvec = torch.empty(self.n_inject, 256, dtype=torch.float32, device=self.device)
        check(self.L.cn_latent_fwd(self._plan, ptr(self.table(params)), ptr(shape_code), ptr(texture_code),
                                   ptr(blob), ptr(zvec), self.stream), "cn_latent_fwd")
        return blob, zvec

    # ------------------------------------------------------------ MLP
    def mlp_fwd(self, blob, M, xyz=None, viewdir=None, rays_o=None, rays_d=None, z=None, z_stride=0,
                n_samples=0, act=None, act_M=0, act_row0=0, sigma=None, rgb=None, codes=False):
        """act_M / act_row0: the workspace is sized for act_M samples and this
        pass fills rows [act_row0, act_row0 + pad(M)) (coarse + fine passes).
        codes: codes-only optimisation -- store only what mlp_bwd(codes=True)
        needs (cn_mlp_fwd_codes)."""
        Mp = self.pad(M)
        if sigma is None:
            sigma = torch.empty(Mp, dtype=torch.float32, device=self.device)
        if rgb is None:
            rgb = torch.empty(Mp, 3, dtype=torch.float32, device=self.device)
        assert sigma.numel() >= Mp and rgb.numel() >= 3 * Mp
        fn = self.L.cn_mlp_fwd_codes if codes else self.L.cn_mlp_fwd
        check(fn(self._plan, ptr(self.pack_fwd), ptr(blob), M, ptr(xyz), ptr(viewdir),
                 ptr(rays_o), ptr(rays_d), ptr(z), z_stride, n_samples, ptr(sigma), ptr(rgb),
                 ptr(act), int(act_M), int(act_row0), self.stream), "cn_mlp_fwd")
        return sigma, rgb

    def new_act(self, M):
        return torch.empty(self.act_bytes(M), dtype=torch.uint8, device=self.device)

    def mlp_bwd(self, blob, M, dsigma, drgb, act, codes=False, act_M=0, row0=0):
        """dX chain over rows [row0, row0 + pad(M)) of an act_M-sample workspace
        (act_M 0: M); dsigma / drgb hold the range's rows.  codes: the
        codes-only variant (stores only the planes mlp_dbias reads)."""
        fn = self.L.cn_mlp_bwd_codes if codes else self.L.cn_mlp_bwd_rows
        check(fn(self._plan, ptr(self.pack_bwd), ptr(blob), M, ptr(dsigma), ptr(drgb), ptr(act), int(act_M),
                 int(row0), self.stream), "cn_mlp_bwd")

    def mlp_dw(self, act, M, zvec, grads, dbuf, ws=None, act_M=0, row0=0, db_accum=False, nwg=0, params=None):
        """Weight gradients over rows [row0, row0 + pad(M)) (grads accumulate;
        dbuf is overwritten, or accumulated with db_accum).  ``grads``: the
        list of gradient tensors or a pointer table from ``table()``;
        nwg: persistent workgroups (0 = one per CU).  The encoding_shape fold
        reads the forward's weights: ``params`` (tensors or a table), default
        the parameters of the last ensure_packed."""
        ptab = self._param_tab if params is None else (
            params if isinstance(params, torch.Tensor) else self.table(params))
        if ptab is None:
            raise RuntimeError("mlp_dw: no packed weights (call ensure_packed before the forward)")
        if ws is None:
            ws = torch.empty(self.dw_ws_bytes(M), dtype=torch.uint8, device=self.device)
        tab = grads if isinstance(grads, torch.Tensor) else self.table(grads)
        # the tables may be used on a stream other than the one they were made on
        cur = torch.cuda.current_stream(self.device)
        tab.record_stream(cur)
        ptab.record_stream(cur)
        check(self.L.cn_mlp_dw_rows(self._plan, ptr(act), int(act_M), int(row0), M, ptr(zvec),
                                    ptr(ptab), ptr(tab), ptr(dbuf), int(bool(db_accum)), int(nwg), ptr(ws),
                                    self.stream), "cn_mlp_dw_rows")

    def mlp_dbias(self, act, M, dbuf, ws=None, act_M=0):
        if ws is None:
            ws = torch.empty(self.dw_ws_bytes(M), dtype=torch.uint8, device=self.device)
        check(self.L.cn_mlp_dbias(self._plan, ptr(act), int(act_M), M, ptr(dbuf), ptr(ws), self.stream),
              "cn_mlp_dbias")

    def latent_bwd(self, params, grads, shape_code, texture_code, zvec, dbuf, d_shape, d_tex, reg_coef=0.0,
                   reg_out=None):
        scratch = torch.empty(self.n_inject, 256, dtype=torch.float32, device=self.device)
        check(self.L.cn_latent_bwd(self._plan, ptr(self.table(params)), ptr(self.table(grads)), ptr(shape_code),
                                   ptr(texture_code), ptr(zvec), ptr(dbuf), ptr(scratch), ptr(d_shape), ptr(d_tex),
                                   float(reg_coef), ptr(reg_out), self.stream), "cn_latent_bwd")


# ---------------------------------------------------------------- rendering
def _dev_stream(t):
    return _lib.stream_ptr(t.device)


def composite_fwd(sigma, rgb, z, R, N, white_bg=True, weights=None):
    L = _lib.lib()
    z_stride = 0 if z.numel() == N else N
    out_rgb = torch.empty(R, 3, dtype=torch.float32, device=sigma.device)
    depth = torch.empty(R, dtype=torch.float32, device=sigma.device)
    check(L.cn_composite_fwd(ptr(sigma), ptr(rgb), ptr(z), z_stride, R, N, int(white_bg), ptr(out_rgb), ptr(depth),
                             ptr(weights), _dev_stream(sigma)), "cn_composite_fwd")
    return out_rgb, depth


def composite_bwd(sigma, rgb, z, R, N, grad_rgb, grad_depth=None, white_bg=True):
    L = _lib.lib()
    z_stride = 0 if z.numel() == N else N
    dsig = torch.empty(R * N, dtype=torch.float32, device=sigma.device)
    drgb = torch.empty(R * N, 3, dtype=torch.float32, device=sigma.device)
    check(L.cn_composite_bwd(ptr(sigma), ptr(rgb), ptr(z), z_stride, R, N, int(white_bg), ptr(grad_rgb),
                             ptr(grad_depth), ptr(dsig), ptr(drgb), _dev_stream(sigma)), "cn_composite_bwd")
    return dsig, drgb


def render_loss(sigma, rgb, z, R, N, gt, chunk, white_bg=True, dsig=None, drgb=None):
    L = _lib.lib()
    dev = sigma.device
    z_stride = 0 if z.numel() == N else N
    out_rgb = torch.empty(R, 3, dtype=torch.float32, device=dev)
    ray_se = torch.empty(R, dtype=torch.float32, device=dev)
    nchunk = (R + chunk - 1) // chunk
    chunk_loss = torch.empty(nchunk, dtype=torch.float32, device=dev)
    if dsig is None:
        dsig = torch.empty(R * N, dtype=torch.float32, device=dev)
    if drgb is None:
        drgb = torch.empty(R * N, 3, dtype=torch.float32, device=dev)
    check(L.cn_render_loss(ptr(sigma), ptr(rgb), ptr(z), z_stride, R, N, int(white_bg), ptr(gt), chunk,
                           ptr(out_rgb), ptr(ray_se), ptr(chunk_loss), ptr(dsig), ptr(drgb), _dev_stream(sigma)),
          "cn_render_loss")
    return out_rgb, chunk_loss, dsig, drgb


def sample_pdf(sigma_c, z_c, R, Nc, rand):
    """Fine z (R, Nf) from the coarse densities; rand (R, Nf) in [0, 1)."""
    L = _lib.lib()
    Nf = rand.shape[-1]
    zc_stride = 0 if z_c.numel() == Nc else Nc
    z_f = torch.empty(R, Nf, dtype=torch.float32, device=sigma_c.device)
    check(L.cn_sample_pdf(ptr(sigma_c), ptr(z_c), zc_stride, R, Nc, ptr(rand), Nf, ptr(z_f),
                          _dev_stream(sigma_c)), "cn_sample_pdf")
    return z_f


def render_loss_fine(sigma_c, rgb_c, z_c, Nc, sigma_f, rgb_f, z_f, Nf, R, gt, chunk, dsig_c, drgb_c,
                     dsig_f, drgb_f, white_bg=True):
    """Fine composite + MSE over the merged samples; accumulates into
    dsig_c / drgb_c, writes dsig_f / drgb_f.  -> (rgb (R,3), chunk losses)."""
    L = _lib.lib()
    dev = sigma_c.device
    zc_stride = 0 if z_c.numel() == Nc else Nc
    out_rgb = torch.empty(R, 3, dtype=torch.float32, device=dev)
    ray_se = torch.empty(R, dtype=torch.float32, device=dev)
    chunk_loss = torch.empty((R + chunk - 1) // chunk, dtype=torch.float32, device=dev)
    check(L.cn_render_loss_fine(ptr(sigma_c), ptr(rgb_c), ptr(z_c), zc_stride, Nc, ptr(sigma_f), ptr(rgb_f),
                                ptr(z_f), Nf, R, int(white_bg), ptr(gt), chunk, ptr(out_rgb), ptr(ray_se),
                                ptr(chunk_loss), ptr(dsig_c), ptr(drgb_c), ptr(dsig_f), ptr(drgb_f),
                                _dev_stream(sigma_c)), "cn_render_loss_fine")
    return out_rgb, chunk_loss


def get_rays_dev(H, W, focal, focal_is_f64, c2w):
    L = _lib.lib()
    dev = c2w.device
    ro = torch.empty(H * W, 3, dtype=torch.float32, device=dev)
    vd = torch.empty(H * W, 3, dtype=torch.float32, device=dev)
    check(L.cn_get_rays(H, W, float(focal), int(focal_is_f64), ptr(c2w), ptr(ro), ptr(vd), _dev_stream(c2w)),
          "cn_get_rays")
    return ro, vd


def sample_points(ro, vd, z, R, N):
    L = _lib.lib()
    z_stride = 0 if z.numel() == N else N
    xyz = torch.empty(R, N, 3, dtype=torch.float32, device=ro.device)
    vrep = torch.empty(R, N, 3, dtype=torch.float32, device=ro.device)
    check(L.cn_sample_points(ptr(ro), ptr(vd), ptr(z), z_stride, R, N, ptr(xyz), ptr(vrep), _dev_stream(ro)),
          "cn_sample_points")
    return xyz, vrep


def adamw_step(params, grads, exp_avgs, exp_avg_sqs, lrs, weight_decay, beta1, beta2, eps, step, zero_grad=False):
    """zero_grad: the kernel also sets every gradient to 0 after reading it."""
    L = _lib.lib()
    n = len(params)
    P = ctypes.c_void_p * n
    keep = []

    def arr(vals, ctype):
        a = (ctype * n)(*vals)
        keep.append(a)
        return ctypes.cast(a, ctypes.c_void_p)

    ptrs = lambda ts: arr([t.data_ptr() for t in ts], ctypes.c_void_p)
    counts = arr([t.numel() for t in params], ctypes.c_int)
    lr = arr([float(x) for x in lrs], ctypes.c_double)
    fn = L.cn_adamw_step_zero_grad if zero_grad else L.cn_adamw_step
    check(fn(n, ptrs(params), ptrs(grads), ptrs(exp_avgs), ptrs(exp_avg_sqs), counts, lr,
             float(weight_decay), float(beta1), float(beta2), float(eps), int(step),
             _dev_stream(params[0])), "cn_adamw_step")
    # the kernel wrote the tensors behind torch's back: bump their version
    # counters so version-keyed caches (the packed weights) see the update
    increment_version(list(params))
    increment_version(list(exp_avgs) + list(exp_avg_sqs))
