"""Torch-CPU restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY.

Written from the reference's behaviour, functionally (a parameter dict keyed by
the reference's state_dict names), so the same arithmetic can be replayed on
the CPU next to the HIP path.  Every function cites the reference lines it
restates.  Pinned by tests/test_oracle.py against tests/golden/*.npz, which
were produced by importing the reference itself (tools/gen_golden.py).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F


def _t(x, dtype=torch.float32):
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x), dtype=dtype)


# ---------------------------------------------------------------- geometry
def get_rays(H, W, focal, c2w):
    """src/utils.py:10-19.  Pixel (row j, col i) -> OpenGL camera ray.

    ``focal`` may be a python float or a float64 tensor of shape (1,) (what
    default_collate makes of the float focal, src/data.py:31-37); in the
    latter case the camera-space directions are formed in float64 and only
    then cast to c2w's dtype, exactly as torch type promotion does in the
    reference.  No +0.5 pixel-centre offset; principal point (W/2, H/2).
    """
    c2w = _t(c2w)
    cols = torch.arange(W, dtype=torch.float32)   # == linspace(0, W-1, W)
    rows = torch.arange(H, dtype=torch.float32)
    jj, ii = torch.meshgrid(rows, cols, indexing="ij")   # (H, W)
    f = focal if isinstance(focal, torch.Tensor) else torch.tensor(float(focal), dtype=torch.float32)
    dx = (ii - W * 0.5) / f
    dy = -(jj - H * 0.5) / f
    cam = torch.stack([dx, dy, -torch.ones_like(dx)], -1).to(c2w.dtype)   # (H, W, 3)
    R = c2w[:3, :3]
    # world dir component a = sum_b cam[b] * R[a, b]  (three products, summed in order)
    prods = cam[..., None, :] * R                       # (H, W, 3, 3)
    d = torch.sum(prods, -1)
    vd = d / torch.norm(d, dim=-1, keepdim=True)
    ro = c2w[:3, 3].expand(d.shape)
    return ro.reshape(-1, 3), vd.reshape(-1, 3)


def stratified_z(near, far, n, jitter=None, z_fixed=False):
    """src/utils.py:24-29.  One z vector shared by all rays.  ``jitter`` is the
    (n,) U[0,1) draw the reference takes with torch.rand(n) (upper half-bin)."""
    if z_fixed:
        return torch.linspace(near, far, n)
    half = (far - near) / (2 * n)
    z = torch.linspace(near + half, far - half, n)
    if jitter is None:
        jitter = torch.rand(n)
    return z + _t(jitter) * (far - near) / (2 * n)


def sample_from_rays(ro, vd, near, far, n, jitter=None, z_fixed=False):
    """src/utils.py:21-32 -> (xyz (R,n,3), viewdir (R,n,3), z (n,))."""
    z = stratified_z(near, far, n, jitter, z_fixed).type_as(ro)
    xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
    return xyz, vd[:, None, :].expand(-1, n, -1).contiguous(), z


# ---------------------------------------------------------------- model
def positional_encoding(x, n_freq):
    """src/model.py:4-7: [x, sin(2^i x)..., cos(2^i x)...], frequency-major,
    component-minor, no pi."""
    scaled = [x * (2.0 ** i) for i in range(n_freq)]
    y = torch.cat(scaled, -1)
    return torch.cat([x, torch.sin(y), torch.cos(y)], -1)


# ---- the bf16 kernels' operand precision, restated (chain.hip / dw.hip with
# CN_BF16): every per-sample Linear multiplies bf16-rounded inputs by
# bf16-rounded weights with fp32 accumulation and an fp32 bias; the backward
# uses bf16-rounded upstream gradients (the stored dA planes) against the
# bf16 weights (dX) and the bf16 inputs (dW).  The per-object latent layers
# and the sigma head run in fp32 there (latent.hip; the sigma head reads the
# fp32 accumulator), so they stay fp32 here.  Off by default: the oracle is
# the fp32 reference; ``bf16_operands()`` switches a block of code over.
#
# ``split_w`` carries every weight as W_hi + W_lo (two bf16, W_hi = rn(W),
# W_lo = rn(W - W_hi)) in the forward and in dX; ``split_x`` / ``split_dy``
# additionally split the layer inputs / upstream gradients the same way.
# The bf16x3 kernels (precision "bf16x3", OPS_BF16X3 below) split weights and
# chain operands and issue three MFMAs per block, hi*hi + hi*lo + lo*hi (the
# dropped lo*lo term is ~2^-16 relative): the sum of the split operands is
# what _q(.., "s") forms.  ``ops`` sets each operand separately, for the
# emulation probes (tools/split_emu.py): keys fw_w, fw_x (forward), bw_w,
# bw_dy (dX), dw_x, dw_dy (dW); values "b" (bf16), "s" (hi + lo), "f" (fp32).
_OPS_BF16 = dict(fw_w="b", fw_x="b", bw_w="b", bw_dy="b", dw_x="b", dw_dy="b")
# the bf16x3 kernels (chain.hip, dw.hip): weights and layer inputs split in
# the forward, weights and upstream gradients split in dX, the dW pass's X
# operands split (the training forward stores their lo parts; encoding_viewdir's
# dir-PE columns stay hi only), its upstream gradients bf16
OPS_BF16X3 = dict(fw_w="s", fw_x="s", bw_w="s", bw_dy="s", dw_x="s", dw_dy="b")
# ... and as the kernels form the latent path's gradient (inj_dy, _lin_inj):
# from the sum of the bf16 dA plane
OPS_BF16X3_DB = dict(OPS_BF16X3, inj_dy="b")
# the kernels' arithmetic op for op (round 5, tools/x3_trace.py): the above,
# plus ``x3`` -- a product of two split operands is hi*hi + hi*lo + lo*hi
# (three MFMAs; the lo*lo term dropped) instead of the exact (hi+lo)(hi+lo) --
# and ``fold`` -- encoding_shape / sigma / encoding_viewdir as the dW pass
# forms their gradients through the encoding_shape fold (_FoldBlock)
OPS_BF16X3_K = dict(OPS_BF16X3_DB, x3=True, fold=True)
# the bf16x3f plan (precision "bf16x3f"): the bf16x3 forward chains (weights
# and layer inputs split, three products) and the bf16 backward (dX and dW on
# bf16 operands, the latent path from the bf16 dA sums)
OPS_BF16X3F = dict(_OPS_BF16, fw_w="s", fw_x="s", x3=True, inj_dy="b")
# the built kernels' per-layer exception: encoding_viewdir's dir-PE columns
# stay hi only in dW (``bf16_operands(ops=..., layer_ops=X3_LAYER_OPS)``)
X3_LAYER_OPS = {"encoding_viewdir.0": {"dw_x_split_cols": 256}}
_BF16 = {"on": False, "ops": dict(_OPS_BF16)}


def _rb(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _rh(t):
    return t.to(torch.float16).to(torch.float32)


def _q(t, how, scale=1.0):
    """t as an operand: "b" bf16-rounded, "s" hi + lo bf16 pair summed in
    fp32 (exact: <= 16 significant bits), "h" fp16-rounded, "hs" hi + lo
    fp16 pair (IEEE fp16 incl. subnormals: ~22 bits in range), "f"
    unchanged.  ``scale`` (a power of two) multiplies t before an fp16
    rounding and divides after (the backward's gradient scale)."""
    if how == "f":
        return t
    if how in ("h", "hs"):
        u = t * scale
        hi = _rh(u)
        r = hi + _rh(u - hi) if how == "hs" else hi
        return r / scale
    hi = _rb(t)
    return hi + _rb(t - hi) if how == "s" else hi


def _split(t):
    hi = _rb(t)
    return hi, _rb(t - hi)


def _mm(a, ha, b, hb, o, gs=1.0):
    """_q(a, ha) @ _q(b, hb), or -- ``o["x3"]`` and both operands split --
    the three products the bf16x3 kernels issue (hi hi + hi lo + lo hi: the
    lo lo term dropped)."""
    if o.get("x3") and ha == "s" and hb == "s" and gs == 1.0:
        ah, al = _split(a)
        bh, bl = _split(b)
        return ah @ bh + (ah @ bl + al @ bh)
    return _q(a, ha, gs) @ _q(b, hb)


class _Bf16Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, o):
        ctx.save_for_backward(x, w)
        ctx.o = o
        return _mm(x, o["fw_x"], w.t(), o["fw_w"], o) + b

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        o = ctx.o
        gs = o.get("grad_scale", 1.0)
        dx = _mm(dy, o["bw_dy"], w, o["bw_w"], o, gs)
        d2 = _q(dy, o["dw_dy"], gs).reshape(-1, dy.shape[-1])
        n = o.get("dw_x_split_cols")       # the kernels: only the leading n columns split
        if n is None:
            x2 = _q(x, o["dw_x"])
        else:
            x2 = torch.cat([_q(x[..., :n], o["dw_x"]), _q(x[..., n:], "b")], -1)
        x2 = x2.reshape(-1, x.shape[-1])
        return dx, d2.t() @ x2, d2.sum(0), None


class bf16_operands:
    """with ref_cpu.bf16_operands(): ... -- the bf16 kernels' arithmetic;
    ``bf16_operands(ops=OPS_BF16X3)`` the bf16x3 kernels'."""

    def __init__(self, split_w=False, split_x=False, split_dy=False, ops=None, layer_ops=None):
        o = dict(_OPS_BF16)
        if split_w:
            o.update(fw_w="s", bw_w="s")
        if split_x:
            o.update(fw_x="s", dw_x="s")
        if split_dy:
            o.update(bw_dy="s", dw_dy="s")
        o.update(ops or {})
        # per-layer overrides (emulation probes): {layer name: {op: how}}
        lo = {k: dict(o, **v) for k, v in (layer_ops or {}).items()}
        self.cfg = {"on": True, "ops": o, "layer_ops": lo}

    def __enter__(self):
        self.prev = {"on": _BF16["on"], "ops": _BF16["ops"], "layer_ops": _BF16.get("layer_ops", {})}
        _BF16.update(self.cfg)

    def __exit__(self, *exc):
        _BF16.update(self.prev)


def _lin(p, name, x):
    if _BF16["on"] and "latent" not in name and not name.startswith("sigma"):
        return _Bf16Linear.apply(x, p[name + ".weight"], p[name + ".bias"],
                                 _BF16.get("layer_ops", {}).get(name, _BF16["ops"]))
    return F.linear(x, p[name + ".weight"], p[name + ".bias"])


class _FoldBlock(torch.autograd.Function):
    """encoding_shape -> (sigma head, encoding_viewdir) as the bf16x3 kernels
    compute it (``ops["fold"]``; chain_set.h / dw.hip):
    forward and dX as _Bf16Linear (the sigma head in fp32 from the fp32
    encoding_shape output); the weight gradients through the encoding_shape
    fold: Gx = sum_s rn(dA_v) (x) [Y_s | 1] (Y_s split, the sigma row from the
    split ds), then d[W_v y-part; w_sigma] = Gx [W_e | b_e]^T and
    d[W_e | b_e] = [W_v; w_sigma]^T Gx in fp32 -- NOT sum rn(dA_e) (x) Y_s,
    the per-layer restatement's encoding_shape gradient."""

    @staticmethod
    def forward(ctx, ys, dpe, We, be, Ws, bs, Wv, bv, oe, ov):
        ye = _mm(ys, oe["fw_x"], We.t(), oe["fw_w"], oe) + be
        spre = F.linear(ye, Ws, bs)
        vpre = _mm(torch.cat([ye, dpe], -1), ov["fw_x"], Wv.t(), ov["fw_w"], ov) + bv
        ctx.save_for_backward(ys, dpe, We, be, Ws, Wv)
        ctx.o = (oe, ov)
        return spre, vpre

    @staticmethod
    def backward(ctx, dspre, dvpre):
        ys, dpe, We, be, Ws, Wv = ctx.saved_tensors
        oe, ov = ctx.o
        F0 = We.shape[0]
        dye = _mm(dvpre, ov["bw_dy"], Wv[:, :F0], ov["bw_w"], ov) + dspre @ Ws
        dys = _mm(dye, oe["bw_dy"], We, oe["bw_w"], oe)
        rA = _q(dvpre, ov["dw_dy"]).reshape(-1, dvpre.shape[-1])
        ysx = _q(ys, oe["dw_x"]).reshape(-1, ys.shape[-1])
        # the sigma-head gradient rides in the viewdir dA plane as value +
        # rounding residual (chain.hip prologue_bwd): split wherever that
        # plane is rounded, exact in an fp32 plan
        dsf = _q(dspre, "f" if ov["dw_dy"] == "f" else "s").reshape(-1, 1)
        # the dir-PE columns of encoding_viewdir's dW operand: dw_x, unless the
        # layer splits only its leading dw_x_split_cols columns (X3_LAYER_OPS:
        # the kernels keep the dir-PE tile hi only) -- then bf16
        n_split = ov.get("dw_x_split_cols")
        how_pe = ov["dw_x"] if n_split is None or n_split > F0 else "b"
        Gx, Gb = rA.t() @ ysx, rA.sum(0)
        Gs, Gsb = dsf.t() @ ysx, dsf.sum(0)
        dWv = torch.cat([Gx @ We.t() + Gb[:, None] * be[None, :],
                         rA.t() @ _q(dpe, how_pe).reshape(-1, dpe.shape[-1])], 1)
        dWs = Gs @ We.t() + Gsb[:, None] * be[None, :]
        dWe = Wv[:, :F0].t() @ Gx + Ws.t() @ Gs
        dbe = Wv[:, :F0].t() @ Gb + Ws[0] * Gsb
        return dys, None, dWe, dbe, dWs, Gsb, dWv, Gb, None, None


class _InjSum(torch.autograd.Function):
    """y + zl with zl (1, F) broadcast over the samples; the backward hands zl
    the sum over samples of the upstream gradient ROUNDED as ``how`` first --
    the kernels' latent path: dz = W^T db and dW += db (x) z with db the sum
    of the stored (bf16) dA plane (dw.hip bias sums), where autograd's
    broadcast would sum the fp32 gradient."""

    @staticmethod
    def forward(ctx, y, zl, how):
        ctx.how = how
        ctx.zshape = zl.shape
        return y + zl

    @staticmethod
    def backward(ctx, dy):
        d = _q(dy, ctx.how).reshape(-1, dy.shape[-1]).sum(0)
        return dy, d.reshape(ctx.zshape), None


def _lin_inj(p, name, h, z):
    """layer `name` applied to h + z (a latent injection).  In the bf16
    emulation as the kernels compute it: the injection is folded into the
    layer's bias in fp32 (latent.hip: b + W z), only h is a bf16 operand; the
    op ``inj_dy`` ("f" default) rounds the upstream gradient of the latent
    path before its sum over samples ("b": the kernels' bias sums)."""
    if _BF16["on"]:
        o = _BF16.get("layer_ops", {}).get(name, _BF16["ops"])
        how = o.get("inj_dy", "f")
        zl = F.linear(z, p[name + ".weight"])
        if how == "f":
            return _lin(p, name, h) + zl
        return _InjSum.apply(_lin(p, name, h), zl, how)
    return _lin(p, name, h + z)


def codenerf_forward(p, xyz, viewdir, shape_code, texture_code, shape_blocks=3,
                     texture_blocks=1, num_xyz_freq=10, num_dir_freq=4, acts=None):
    """src/model.py:36-53.  Returns (sigmas (...,1), rgbs (...,3)).

    Latent injection: y <- y + ReLU(L_j code + c_j) before every shape /
    texture layer; encoding_shape has no activation; sigma = Softplus(beta=1,
    threshold=20); the rgb head is linear (no sigmoid).  ``acts`` (a dict)
    optionally receives every intermediate for per-layer checks.
    """
    h = F.relu(_lin(p, "encoding_xyz.0", positional_encoding(xyz, num_xyz_freq)))
    if acts is not None:
        acts["y0"] = h
    for j in range(1, shape_blocks + 1):
        z = F.relu(_lin(p, f"shape_latent_layer_{j}.0", shape_code))
        h = F.relu(_lin_inj(p, f"shape_layer_{j}.0", h, z))
        if acts is not None:
            acts[f"y{j}"] = h
    # (the fold computes encoding_shape's output inside _FoldBlock: a call
    # asking for the per-layer activations runs the per-layer restatement)
    if _BF16["on"] and _BF16["ops"].get("fold") and acts is None:
        lo = _BF16.get("layer_ops", {})
        dpe = positional_encoding(viewdir, num_dir_freq)
        spre, vpre = _FoldBlock.apply(h, dpe, p["encoding_shape.weight"], p["encoding_shape.bias"],
                                      p["sigma.0.weight"], p["sigma.0.bias"], p["encoding_viewdir.0.weight"],
                                      p["encoding_viewdir.0.bias"], lo.get("encoding_shape", _BF16["ops"]),
                                      lo.get("encoding_viewdir.0", _BF16["ops"]))
        sig = F.softplus(spre, beta=1.0, threshold=20.0)
        h = F.relu(vpre)
    else:
        h = _lin(p, "encoding_shape", h)
        if acts is not None:
            acts["y_shape"] = h
        sig = F.softplus(_lin(p, "sigma.0", h), beta=1.0, threshold=20.0)
        h = F.relu(_lin(p, "encoding_viewdir.0",
                        torch.cat([h, positional_encoding(viewdir, num_dir_freq)], -1)))
    if acts is not None:
        acts["y_view"] = h
    for j in range(1, texture_blocks + 1):
        z = F.relu(_lin(p, f"texture_latent_layer_{j}.0", texture_code))
        h = F.relu(_lin_inj(p, f"texture_layer_{j}.0", h, z))
        if acts is not None:
            acts[f"y_tex{j}"] = h
    h = F.relu(_lin(p, "rgb.0", h))
    if acts is not None:
        acts["y_rgb0"] = h
    return sig, _lin(p, "rgb.2", h)


# ---------------------------------------------------------------- rendering
def volume_rendering(sigmas, rgbs, z_vals, white_bg=True):
    """src/utils.py:34-47.  Alpha compositing along the sample axis.

    z_vals may be (N,) (shared, as the reference) or (R,N) (per ray, used by
    the fine-sampling extension).  The last interval is 1e10; transmittance
    is the exclusive cumulative product of (1 - alpha + 1e-10).
    """
    sig = sigmas[..., 0] if sigmas.dim() == 3 else sigmas
    gaps = z_vals[..., 1:] - z_vals[..., :-1]
    gaps = torch.cat([gaps, torch.full_like(gaps[..., :1], 1e10)], -1)
    alpha = 1 - torch.exp(-sig * gaps)
    keep = 1 - alpha + 1e-10
    T = torch.cumprod(torch.cat([torch.ones_like(keep[..., :1]), keep], -1), -1)[..., :-1]
    w = alpha * T
    rgb = torch.sum(w[..., None] * rgbs, -2)
    depth = torch.sum(w * z_vals, -1)
    if white_bg:
        rgb = rgb + 1 - w.sum(1)[..., None]
    return rgb, depth


# ---------------------------------------------------------------- training
def param_tensors(np_params, requires_grad=True):
    return {k: torch.tensor(v, requires_grad=requires_grad) for k, v in np_params.items()}


def image_step(p, shape_table, texture_table, obj_idx, ro, vd, z_vals, gt, chunk=2048,
               reg_coef=1e-4, net=None):
    """One image of the training loop, src/trainer.py:65-84.

    Chunks of ``chunk`` rays: per-chunk mean MSE, ``loss.backward()`` per
    chunk (so gradients are the sum of chunk-mean gradients) and the code
    regulariser ``reg_coef * mean(|s| + |t|)`` added on chunk 0 only.
    ``p`` / tables must be leaf tensors with requires_grad; gradients are
    accumulated into ``.grad``.  Returns (per-chunk l2 losses, rgb image).
    """
    net = net or {}
    n = z_vals.shape[-1]
    R = ro.shape[0]
    losses, outs = [], []
    for a in range(0, R, chunk):
        b = min(a + chunk, R)
        s = shape_table[obj_idx][None]
        t = texture_table[obj_idx][None]
        zc = z_vals if z_vals.dim() == 1 else z_vals[a:b]
        xyz = ro[a:b, None, :] + vd[a:b, None, :] * zc[..., None]
        vdir = vd[a:b, None, :].expand(-1, n, -1)
        sig, rgbs = codenerf_forward(p, xyz, vdir, s, t, **net)
        rgb, _ = volume_rendering(sig, rgbs, zc)
        l2 = torch.mean((rgb - gt[a:b]) ** 2)
        loss = l2
        if a == 0:
            loss = l2 + reg_coef * torch.mean(torch.norm(s, dim=-1) + torch.norm(t, dim=-1))
        loss.backward()
        losses.append(l2.item())
        outs.append(rgb.detach())
    return losses, torch.cat(outs)


# ---------------------------------------------------------------- fine pass
# The BASELINE configs' "64 coarse + 64 fine" has no counterpart in the
# reference (one stratified pass only, src/utils.py:21-32; SURVEY.md section
# 0): these restate NeRF's hierarchical sampling as the HIP path defines it
# (include/codenerf.h cn_sample_pdf / cn_render_loss_fine).  PARITY UNPINNED:
# no reference output exists; they check the HIP kernels' self-consistency.
def composite_weights(sigmas, z_vals):
    """The weights alpha * T of volume_rendering (src/utils.py:36-42)."""
    sig = sigmas[..., 0] if sigmas.dim() == 3 else sigmas
    gaps = z_vals[..., 1:] - z_vals[..., :-1]
    gaps = torch.cat([gaps, torch.full_like(gaps[..., :1], 1e10)], -1)
    alpha = 1 - torch.exp(-sig * gaps)
    keep = 1 - alpha + 1e-10
    T = torch.cumprod(torch.cat([torch.ones_like(keep[..., :1]), keep], -1), -1)[..., :-1]
    return alpha * T


def sample_pdf(sigmas, z_vals, rand):
    """Importance samples (R, Nf): bins = coarse-z midpoints, pdf = w[1:-1] +
    1e-5 normalised, cdf = [0, cumsum] (float64, rounded once), stratified
    u_j = (j + rand_j) / Nf, inverse cdf with NeRF's degenerate-bin rule."""
    R, Nc = sigmas.shape[0], sigmas.shape[-1] if sigmas.dim() == 2 else sigmas.shape[1]
    sig = sigmas.reshape(R, Nc)
    z = z_vals.expand(R, Nc) if z_vals.dim() == 1 else z_vals
    w = composite_weights(sig, z)[:, 1:-1] + 1e-5
    cs = torch.cumsum(w.double(), -1)
    cdf = torch.cat([torch.zeros(R, 1, dtype=torch.float32, device=sig.device), (cs / cs[:, -1:]).float()], -1)   # (R, Nc-1)
    bins = 0.5 * (z[:, :-1] + z[:, 1:])
    Nf = rand.shape[-1]
    u = (torch.arange(Nf, dtype=torch.float32, device=rand.device)[None, :] + rand) / Nf
    inds = torch.searchsorted(cdf, u.contiguous(), right=True)
    below = torch.clamp(inds - 1, min=0)
    above = torch.clamp(inds, max=Nc - 2)
    cb, ca = torch.gather(cdf, 1, below), torch.gather(cdf, 1, above)
    bb, ba = torch.gather(bins, 1, below), torch.gather(bins, 1, above)
    denom = ca - cb
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cb) / denom
    return bb + t * (ba - bb)


def merge_samples(z_c, z_f, *vals):
    """Union of coarse (R,Nc) and fine (R,Nf) samples sorted by z, a coarse
    sample first at equal z; vals are (coarse, fine) pairs gathered alike."""
    R = z_f.shape[0]
    zc = z_c.expand(R, -1) if z_c.dim() == 1 else z_c
    z = torch.cat([zc, z_f], -1)
    z_sorted, order = torch.sort(z, dim=-1, stable=True)
    out = [z_sorted]
    for vc, vf in vals:
        v = torch.cat([vc, vf], 1)
        idx = order.reshape(order.shape + (1,) * (v.dim() - 2)).expand(order.shape + v.shape[2:])
        out.append(torch.gather(v, 1, idx))
    return out


def fine_image_step(p, shape_table, texture_table, obj_idx, ro, vd, z_c, z_f, gt, chunk=2048,
                    reg_coef=1e-4, net=None):
    """Coarse + fine training image (HIP: render.ImageStep.forward_backward_fine):
    per chunk, loss = mean MSE of the coarse composite + mean MSE of the
    composite over the merged coarse and fine samples (+ the code regulariser
    on chunk 0), backward per chunk.  z_f (R, Nf) is given (from sample_pdf).
    Returns (coarse losses, fine losses, fine rgb)."""
    net = net or {}
    Nc, Nf = z_c.shape[-1], z_f.shape[-1]
    R = ro.shape[0]
    lc_all, lf_all, outs = [], [], []
    for a in range(0, R, chunk):
        b = min(a + chunk, R)
        s = shape_table[obj_idx][None]
        t = texture_table[obj_idx][None]
        zc = z_c if z_c.dim() == 1 else z_c[a:b]
        xyz = ro[a:b, None, :] + vd[a:b, None, :] * zc[..., None]
        sig_c, rgb_c = codenerf_forward(p, xyz, vd[a:b, None, :].expand(-1, Nc, -1), s, t, **net)
        rgb, _ = volume_rendering(sig_c, rgb_c, zc)
        l2c = torch.mean((rgb - gt[a:b]) ** 2)
        zf = z_f[a:b]
        xyz_f = ro[a:b, None, :] + vd[a:b, None, :] * zf[..., None]
        sig_f, rgb_f = codenerf_forward(p, xyz_f, vd[a:b, None, :].expand(-1, Nf, -1), s, t, **net)
        z_m, sig_m, rgb_m = merge_samples(zc, zf, (sig_c[..., 0], sig_f[..., 0]), (rgb_c, rgb_f))
        rgb2, _ = volume_rendering(sig_m, rgb_m, z_m)
        l2f = torch.mean((rgb2 - gt[a:b]) ** 2)
        loss = l2c + l2f
        if a == 0:
            loss = loss + reg_coef * torch.mean(torch.norm(s, dim=-1) + torch.norm(t, dim=-1))
        loss.backward()
        lc_all.append(l2c.item())
        lf_all.append(l2f.item())
        outs.append(rgb2.detach())
    return lc_all, lf_all, torch.cat(outs)


class AdamWRef:
    """torch.optim.AdamW defaults as used at src/trainer.py:116-120
    (betas 0.9/0.999, eps 1e-8, weight_decay 0.01, no amsgrad), restated in
    the single-tensor update order so it can be mirrored elementwise."""

    def __init__(self, groups, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.groups = groups          # [(list_of_tensors, lr)]
        self.b1, self.b2 = betas
        self.eps, self.wd = eps, weight_decay
        self.state = {}

    @torch.no_grad()
    def step(self):
        for params, lr in self.groups:
            for p in params:
                if p.grad is None:
                    continue
                st = self.state.setdefault(id(p), [0, torch.zeros_like(p), torch.zeros_like(p)])
                st[0] += 1
                step, m, v = st
                p.mul_(1 - lr * self.wd)
                m.lerp_(p.grad, 1 - self.b1)
                v.mul_(self.b2).addcmul_(p.grad, p.grad, value=1 - self.b2)
                bc1 = 1 - self.b1 ** step
                bc2 = 1 - self.b2 ** step
                denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
                p.addcdiv_(m, denom, value=-(lr / bc1))


def psnr(mse):
    """src/trainer.py:99."""
    return -10.0 * np.log(mse) / np.log(10.0)
