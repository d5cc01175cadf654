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
    def __init__(self, model, chunk=2048, reg_coef=1e-4, white_bg=True, timers=None, overlap_dw=True):
        self.model = model
        # coarse + fine step: weight gradients of the fine rows on a second
        # stream while the dX chain runs over the coarse rows
        self.overlap_dw = bool(overlap_dw)
        self._side = None
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
                         reg=True, weight_grads=True):
        """One image: returns (chunk losses [ceil(R/chunk)], rendered rgb [R,3],
        reg loss [1]).  Gradients are accumulated into .grad.  weight_grads
        False (codes-only optimisation, src/optimizer.py): the weight-gradient
        pass is replaced by the bias sums the code gradients need."""
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
                                 n_samples=N, act=buf["act"], codes=not weight_grads)
        if tm:
            tm.done("fwd", ev)
        out_rgb, chunk_loss, dsig, drgb = _eng.render_loss(sigma, rgb, z, R, N, gt, self.chunk, self.white_bg)
        ev = tm.mark("bwd") if tm else None
        eng.mlp_bwd(blob, M, dsig, drgb, buf["act"], codes=not weight_grads)
        if tm:
            tm.done("bwd", ev)
            ev = tm.mark("dw")
        if weight_grads:
            eng.mlp_dw(buf["act"], M, zvec, grads, buf["dbuf"], buf["dw"])
        else:
            eng.mlp_dbias(buf["act"], M, buf["dbuf"], buf["dw"])
            grads = buf.setdefault("scratch_grads", [torch.zeros_like(p) for p in params])
        if tm:
            tm.done("dw", ev)
        reg_out = torch.zeros(1, dtype=torch.float32, device=eng.device)
        eng.latent_bwd(params, grads, s, t, zvec, buf["dbuf"], shape_table.grad[obj_idx],
                       texture_table.grad[obj_idx], self.reg_coef if reg else 0.0, reg_out)
        return chunk_loss, out_rgb, reg_out

    def forward_backward_fine(self, rays_o, viewdirs, z_c, rand_f, gt, shape_table, texture_table, obj_idx,
                              reg=True):
        """Coarse + fine image step (the BASELINE configs' "64 + 64"; no
        reference counterpart -- NeRF hierarchical sampling through the one
        CodeNeRF MLP, oracle/ref_cpu.py:fine_image_step).  Loss = coarse
        chunk-mean MSE + fine chunk-mean MSE (+ code regulariser once).  The
        coarse pass fills activation rows [0, pad(R*Nc)), the fine pass the
        rows after, so one backward and one dW cover both.
        Returns (coarse chunk losses, fine chunk losses, fine rgb (R,3), reg)."""
        model = self.model
        eng = model.engine()
        params = model.param_list()
        grads = self.ensure_grads(params)
        self.ensure_grads([shape_table, texture_table])
        R = rays_o.shape[0]
        Nc = z_c.shape[-1]
        Nf = rand_f.shape[-1]
        Mc, Mf = R * Nc, R * Nf
        Mc_p = eng.pad(Mc)
        M = Mc_p + Mf
        Mp = eng.pad(M)
        z_c = z_c.contiguous().to(eng.device, torch.float32)
        buf = self._buffers(eng, M)
        if "sig" not in buf:
            buf.update(sig=torch.empty(Mp, dtype=torch.float32, device=eng.device),
                       rgb=torch.empty(Mp, 3, dtype=torch.float32, device=eng.device),
                       dsig=torch.empty(Mp, dtype=torch.float32, device=eng.device),
                       drgb=torch.empty(Mp, 3, dtype=torch.float32, device=eng.device))
        sig, rgb, dsig, drgb = buf["sig"], buf["rgb"], buf["dsig"], buf["drgb"]
        dsig.zero_()
        drgb.zero_()
        eng.ensure_packed(params, bwd=True)
        s, t = shape_table.detach()[obj_idx], texture_table.detach()[obj_idx]
        blob, zvec = eng.latent_fwd(params, s, t)
        tm = self.timers
        ev = tm.mark("fwd") if tm else None
        sig_c, rgb_c = eng.mlp_fwd(blob, Mc, rays_o=rays_o, rays_d=viewdirs, z=z_c,
                                   z_stride=0 if z_c.dim() == 1 else Nc, n_samples=Nc, act=buf["act"], act_M=M,
                                   act_row0=0, sigma=sig[:Mc_p], rgb=rgb[:Mc_p])
        if tm:
            tm.done("fwd", ev)
        _, loss_c, _, _ = _eng.render_loss(sig_c, rgb_c, z_c, R, Nc, gt, self.chunk, self.white_bg,
                                           dsig=dsig[:Mc], drgb=drgb[:Mc])
        z_f = _eng.sample_pdf(sig_c, z_c, R, Nc, rand_f)
        ev = tm.mark("fwd") if tm else None
        sig_f, rgb_f = eng.mlp_fwd(blob, Mf, rays_o=rays_o, rays_d=viewdirs, z=z_f, z_stride=Nf, n_samples=Nf,
                                   act=buf["act"], act_M=M, act_row0=Mc_p, sigma=sig[Mc_p:], rgb=rgb[Mc_p:])
        if tm:
            tm.done("fwd", ev)
        out_f, loss_f = _eng.render_loss_fine(sig_c, rgb_c, z_c, Nc, sig_f, rgb_f, z_f, Nf, R, gt, self.chunk,
                                              dsig[:Mc], drgb[:Mc], dsig[Mc_p:Mc_p + Mf],
                                              drgb[Mc_p:Mc_p + Mf], self.white_bg)
        if self.overlap_dw:
            self._bwd_dw_overlapped(eng, blob, buf, dsig, drgb, zvec, grads, Mc, Mc_p, Mf, M)
        else:
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
        self.last_z_f = z_f
        return loss_c, loss_f, out_f, reg_out

    def _bwd_dw_overlapped(self, eng, blob, buf, dsig, drgb, zvec, grads, Mc, Mc_p, Mf, M):
        """dX chain over the fine rows, then (current stream) the dX chain over
        the coarse rows while (side stream) dW reduces the fine rows, then dW
        of the coarse rows.  Same rows and sums as one mlp_bwd + mlp_dw over
        [0, M); the fp32 partial order differs.  dW is HBM-bound (operand
        stream), the dX chain MFMA-bound, so the two share the chip."""
        tm = self.timers
        act = buf["act"]
        main = torch.cuda.current_stream(eng.device)
        if self._side is None:
            self._side = torch.cuda.Stream(eng.device)
        side = self._side
        ev = tm.mark("bwd") if tm else None
        eng.mlp_bwd_rows(blob, Mf, dsig[Mc_p:], drgb[Mc_p:], act, M, Mc_p)
        fine_done = torch.cuda.Event()
        fine_done.record(main)
        side.wait_event(fine_done)
        eng.mlp_bwd_rows(blob, Mc, dsig, drgb, act, M, 0)
        if tm:
            tm.done("bwd", ev)
        coarse_done = torch.cuda.Event()
        coarse_done.record(main)
        with torch.cuda.stream(side):
            # timers: one span per dW launch, each from the moment its rows are
            # ready (and the side stream free) to its end
            ev = tm.mark("dw") if tm else None
            eng.mlp_dw_rows(act, M, Mc_p, Mf, zvec, grads, buf["dbuf"], buf["dw"], db_accum=False)
            if tm:
                tm.done("dw", ev)
            side.wait_event(coarse_done)
            ev = tm.mark("dw") if tm else None
            eng.mlp_dw_rows(act, M, 0, Mc, zvec, grads, buf["dbuf"], buf["dw"], db_accum=True)
            if tm:
                tm.done("dw", ev)
        main.wait_stream(side)

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
