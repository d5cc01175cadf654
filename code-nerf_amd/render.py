"""Fused training / rendering steps over whole images.

``ImageStep`` replaces the per-image body of the reference training loop
(src/trainer.py:65-84, and its twin src/optimizer.py:75-94): rays -> samples
-> CodeNeRF -> compositing -> chunk-mean MSE (+ code regulariser on chunk 0)
-> backward into ``.grad`` of the model parameters and the code rows.  The
reference processes 2048-ray chunks with a host sync per chunk; here the whole
image is one pass of five launches, with the chunk semantics of the loss
(gradient = sum of chunk-mean gradients, regulariser counted once) kept
exactly.  Samples are generated inside the MLP kernel from (ray, z); xyz is
never materialised.
"""
import torch

from . import engine as _eng


class ImageStep:
    def __init__(self, model, chunk=2048, reg_coef=1e-4, white_bg=True, timers=None):
        self.model = model
        self.timers = timers
        self.chunk = int(chunk)
        self.reg_coef = float(reg_coef)
        self.white_bg = bool(white_bg)
        self._ws = {}

    def _buffers(self, eng, M):
        b = self._ws.get(M)
        if b is None:
            if len(self._ws) > 4:
                self._ws.clear()
            b = dict(act=eng.new_act(M),
                     dw=torch.empty(eng.dw_ws_bytes(M), dtype=torch.uint8, device=eng.device),
                     dbuf=torch.empty(eng.n_inject, 256, dtype=torch.float32, device=eng.device))
            self._ws[M] = b
        return b

    @staticmethod
    def ensure_grads(tensors):
        for p in tensors:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        return [p.grad for p in tensors]

    def forward_backward(self, rays_o, viewdirs, z_vals, gt, shape_table, texture_table, obj_idx,
                         reg=True):
        """One image: returns (chunk losses [ceil(R/chunk)], rendered rgb [R,3],
        reg loss [1]).  Gradients are accumulated into .grad."""
        model = self.model
        eng = model.engine()
        params = model.param_list()
        grads = self.ensure_grads(params)
        self.ensure_grads([shape_table, texture_table])
        R = rays_o.shape[0]
        N = z_vals.shape[-1]
        M = R * N
        z = z_vals.contiguous().to(eng.device, torch.float32)
        z_stride = 0 if z.dim() == 1 else N
        buf = self._buffers(eng, M)
        eng.ensure_packed(params, bwd=True)
        s, t = shape_table.detach()[obj_idx], texture_table.detach()[obj_idx]
        blob, zvec = eng.latent_fwd(params, s, t)
        tm = self.timers
        ev = tm.mark("fwd") if tm else None
        sigma, rgb = eng.mlp_fwd(blob, M, rays_o=rays_o, rays_d=viewdirs, z=z, z_stride=z_stride,
                                 n_samples=N, act=buf["act"])
        if tm:
            tm.done("fwd", ev)
        out_rgb, chunk_loss, dsig, drgb = _eng.render_loss(sigma, rgb, z, R, N, gt, self.chunk, self.white_bg)
        ev = tm.mark("bwd") if tm else None
        eng.mlp_bwd(blob, M, dsig, drgb, buf["act"])
        if tm:
            tm.done("bwd", ev)
            ev = tm.mark("dw")
        eng.mlp_dw(buf["act"], M, zvec, grads, buf["dbuf"], buf["dw"])
        if tm:
            tm.done("dw", ev)
        reg_out = torch.zeros(1, dtype=torch.float32, device=eng.device)
        eng.latent_bwd(params, grads, s, t, zvec, buf["dbuf"], shape_table.grad[obj_idx],
                       texture_table.grad[obj_idx], self.reg_coef if reg else 0.0, reg_out)
        return chunk_loss, out_rgb, reg_out

    @torch.no_grad()
    def render(self, rays_o, viewdirs, z_vals, shape_code, texture_code):
        """Forward only (src/optimizer.py:108-124): -> rgb (R,3), depth (R,)."""
        eng = self.model.engine()
        params = self.model.param_list()
        R = rays_o.shape[0]
        N = z_vals.shape[-1]
        z = z_vals.contiguous().to(eng.device, torch.float32)
        eng.ensure_packed(params, bwd=False)
        blob, _ = eng.latent_fwd(params, shape_code.reshape(-1).contiguous(), texture_code.reshape(-1).contiguous())
        sigma, rgb = eng.mlp_fwd(blob, R * N, rays_o=rays_o, rays_d=viewdirs, z=z,
                                 z_stride=0 if z.dim() == 1 else N, n_samples=N)
        return _eng.composite_fwd(sigma, rgb, z, R, N, self.white_bg)
