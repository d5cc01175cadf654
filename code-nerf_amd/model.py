"""CodeNeRF on the MI355X chain kernels.

Drop-in for the reference module (src/model.py:10-53): same constructor
arguments, same sub-module / parameter names (so ``state_dict`` round-trips
with the reference's ``models.pth``: src/trainer.py:166-170), same
``forward(xyz, viewdir, shape_latent, texture_latent) -> (sigmas, rgbs)``.
The forward and its backward run as single fused HIP launches (chain.hip)
plus a per-object latent kernel and a weight-gradient pass (dw.hip); nothing
is computed by torch ops (the positional encoding of src/model.py:4-7 is
computed inside the chain kernel).
"""
import torch
import torch.nn as nn

from .engine import Engine



def _linear_block(n_in, n_out, relu):
    mods = [nn.Linear(n_in, n_out)]
    if relu:
        mods.append(nn.ReLU())
    return nn.Sequential(*mods)


class CodeNeRF(nn.Module):
    """Code-conditioned NeRF MLP (reference src/model.py:10-34).

    Extra keyword ``precision`` selects the kernel arithmetic: "fp32" (exact
    fp32 MFMA, parity with the reference), "bf16" (bf16 operands, fp32
    accumulation, throughput), "bf16x3" (every chain operand and weight as a
    bf16 hi + lo pair, three MFMAs per block; dW on hi + lo X operands) or
    "bf16x3f" (the bf16x3 forward -- rendered rgb at fp32 class -- with the
    bf16 backward).

    """

    def __init__(self, shape_blocks=2, texture_blocks=1, W=256, num_xyz_freq=10, num_dir_freq=4,
                 latent_dim=256, precision="fp32"):
        super().__init__()
        self.shape_blocks = shape_blocks
        self.texture_blocks = texture_blocks
        self.num_xyz_freq = num_xyz_freq
        self.num_dir_freq = num_dir_freq
        self.precision = precision
        self.net_cfg = dict(shape_blocks=shape_blocks, texture_blocks=texture_blocks, W=W,
                            num_xyz_freq=num_xyz_freq, num_dir_freq=num_dir_freq, latent_dim=latent_dim)
        d_xyz, d_dir = 3 + 6 * num_xyz_freq, 3 + 6 * num_dir_freq
        # registration order == reference state_dict order
        self.encoding_xyz = _linear_block(d_xyz, W, True)
        for j in range(1, shape_blocks + 1):
            setattr(self, f"shape_latent_layer_{j}", _linear_block(latent_dim, W, True))
            setattr(self, f"shape_layer_{j}", _linear_block(W, W, True))
        self.encoding_shape = nn.Linear(W, W)
        self.sigma = nn.Sequential(nn.Linear(W, 1), nn.Softplus())
        self.encoding_viewdir = _linear_block(W + d_dir, W, True)
        for j in range(1, texture_blocks + 1):
            setattr(self, f"texture_latent_layer_{j}", _linear_block(latent_dim, W, True))
            setattr(self, f"texture_layer_{j}", _linear_block(W, W, True))
        self.rgb = nn.Sequential(nn.Linear(W, W // 2), nn.ReLU(), nn.Linear(W // 2, 3))

    def param_list(self):
        return [p for _, p in self.named_parameters()]

    def engine(self):
        """This module's plan + packed weights (one per module and device:
        the packed blobs are tied to these parameter tensors)."""
        dev = next(self.parameters()).device
        eng = self.__dict__.get("_engine")
        if eng is None or eng.device != dev:
            eng = Engine(precision=self.precision, device=dev, **self.net_cfg)
            self.__dict__["_engine"] = eng
        return eng

    def forward(self, xyz, viewdir, shape_latent, texture_latent):
        params = self.param_list()
        if not params[0].is_cuda:
            raise RuntimeError("CodeNeRF (MI355X) runs on the HIP device only: call .to('cuda') first")
        return _CodeNeRFFunction.apply(self.engine(), xyz, viewdir, shape_latent, texture_latent, *params)


class _CodeNeRFFunction(torch.autograd.Function):
    """One fused launch for the forward (plus the latent layers); the backward
    is the dX chain + weight-gradient pass + latent backward.  A call whose
    training workspace would exceed the activation budget (engine.ACT_BUDGET)
    keeps no activations: its forward runs in inference parts and its
    backward recomputes each part's forward before back-propagating it
    (gradients of the parts accumulate)."""

    @staticmethod
    def forward(ctx, eng, xyz, viewdir, shape_code, texture_code, *params):
        if xyz.shape[-1] != 3 or viewdir.shape != xyz.shape:
            raise ValueError(f"xyz and viewdir must have the same (..., 3) shape, got {tuple(xyz.shape)} "
                             f"and {tuple(viewdir.shape)}")
        if xyz.requires_grad or viewdir.requires_grad:
            raise NotImplementedError("gradients w.r.t. sample positions are not provided (the reference never "
                                      "uses them)")
        lead = xyz.shape[:-1]
        dev = eng.device
        x = xyz.to(dev, torch.float32).contiguous().reshape(-1, 3)
        v = viewdir.to(dev, torch.float32).contiguous().reshape(-1, 3)
        s = shape_code.to(dev, torch.float32).contiguous().reshape(-1)
        t = texture_code.to(dev, torch.float32).contiguous().reshape(-1)
        if s.numel() != 256 or t.numel() != 256:
            raise ValueError("one shape and one texture code of 256 values per call (src/model.py:41-42)")
        M = x.shape[0]
        ctx.eng, ctx.M, ctx.lead = eng, M, lead
        ctx.code_shapes = (shape_code.shape, texture_code.shape)
        if M == 0:
            # empty batch (as torch's nn.Linear: empty outputs, zero gradients)
            ctx.part = -1
            ctx.param_shapes = [p.shape for p in params]
            return (torch.empty(*lead, 1, dtype=torch.float32, device=dev),
                    torch.empty(*lead, 3, dtype=torch.float32, device=dev))
        eng.ensure_packed(params, bwd=True)
        blob, zvec = eng.latent_fwd(params, s, t)
        need_grad = any(ctx.needs_input_grad[3:])
        part = eng.max_act_samples()
        if need_grad and M <= part:
            act = eng.new_act(M)
            sigma, rgb = eng.mlp_fwd(blob, M, xyz=x, viewdir=v, act=act)
            ctx.part = 0
            ctx.save_for_backward(s, t, blob, zvec, act, *params)
            return sigma[:M].reshape(*lead, 1), rgb[:M].reshape(*lead, 3)
        # inference launches over parts (no workspace)
        step = eng.L.cn_max_samples() // 256 * 256
        sigma = torch.empty(M, dtype=torch.float32, device=dev)
        rgb = torch.empty(M, 3, dtype=torch.float32, device=dev)
        for a in range(0, M, step):
            b = min(a + step, M)
            sg, rg = eng.mlp_fwd(blob, b - a, xyz=x[a:b], viewdir=v[a:b])
            sigma[a:b] = sg[:b - a]
            rgb[a:b] = rg[:b - a]
        if need_grad:
            ctx.part = part
            ctx.save_for_backward(s, t, blob, zvec, x, v, *params)
        return sigma.reshape(*lead, 1), rgb.reshape(*lead, 3)

    @staticmethod
    def backward(ctx, g_sigma, g_rgb):
        eng, M = ctx.eng, ctx.M
        if ctx.part == -1:
            z = lambda shp: torch.zeros(shp, dtype=torch.float32, device=eng.device)
            return (None, None, None, z(ctx.code_shapes[0]), z(ctx.code_shapes[1]), *[z(s) for s in ctx.param_shapes])
        dsig = (torch.zeros(M, device=eng.device) if g_sigma is None
                else g_sigma.contiguous().reshape(-1).to(torch.float32))
        drgb = (torch.zeros(M, 3, device=eng.device) if g_rgb is None
                else g_rgb.contiguous().reshape(-1, 3).to(torch.float32))
        dbuf = torch.empty(eng.n_inject, 256, dtype=torch.float32, device=eng.device)
        if ctx.part == 0:
            s, t, blob, zvec, act, *params = ctx.saved_tensors
            grads = [torch.zeros_like(p) for p in params]
            eng.mlp_bwd(blob, M, dsig, drgb, act)
            eng.mlp_dw(act, M, zvec, grads, dbuf, params=params)
        else:
            # recompute each part's forward into one part-sized workspace
            s, t, blob, zvec, x, v, *params = ctx.saved_tensors
            grads = [torch.zeros_like(p) for p in params]
            gtab = eng.table(grads)
            P = ctx.part
            act = eng.new_act(P)
            ws = torch.empty(eng.dw_ws_bytes(P), dtype=torch.uint8, device=eng.device)
            for k, a in enumerate(range(0, M, P)):
                b = min(a + P, M)
                eng.mlp_fwd(blob, b - a, xyz=x[a:b], viewdir=v[a:b], act=act, act_M=P)
                eng.mlp_bwd(blob, b - a, dsig[a:b], drgb[a:b], act, act_M=P)
                eng.mlp_dw(act, b - a, zvec, gtab, dbuf, ws, act_M=P, db_accum=k > 0, params=params)
        ds = torch.zeros(256, dtype=torch.float32, device=eng.device)
        dt = torch.zeros(256, dtype=torch.float32, device=eng.device)
        eng.latent_bwd(params, grads, s, t, zvec, dbuf, ds, dt)
        return (None, None, None, ds.reshape(ctx.code_shapes[0]), dt.reshape(ctx.code_shapes[1]), *grads)
