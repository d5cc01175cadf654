"""Fused training / rendering steps over whole images.

``ImageStep`` replaces the per-image body of the reference training loop
(src/trainer.py:65-84, and its twin src/optimizer.py:75-94): rays -> samples
-> CodeNeRF -> compositing -> chunk-mean MSE (+ code regulariser on chunk 0)
-> backward into ``.grad`` of the model parameters and the code rows.  The
reference processes 2048-ray chunks with a host sync per chunk; here an image
is rendered in as few launches as the activation budget allows, with the
chunk semantics of the loss (gradient = sum of chunk-mean gradients,
regulariser counted once) kept exactly.  Samples are generated inside the MLP
kernel from (ray, z); xyz is never materialised.

Large images (C5: 256^2 rays x 256 samples in fp32) are split into ray parts
of whole loss chunks whose training workspace fits ``engine.ACT_BUDGET``;
their gradients accumulate before the caller's optimiser step.

Backward schedule: the rows of a part (coarse rows, then fine rows) are cut
into ``bwd_ranges`` row ranges; the dX chain of range i runs on the current
stream while the weight-gradient pass of range i-1 runs on a side stream
(the dX chain is MFMA-bound, dW streams its operand planes from HBM).
"""
import ctypes

import torch

from . import _lib
from . import dp as _dp
from . import engine as _eng
from ._lib import check


class ImageStep:
    def __init__(self, model, chunk=2048, reg_coef=1e-4, white_bg=True, timers=None, overlap_dw=True,
                 bwd_ranges=2, dw_side_wgs=0, act_budget=None, max_rays=None):
        self.model = model
        self.timers = timers
        self.chunk = int(chunk)
        self.reg_coef = float(reg_coef)
        self.white_bg = bool(white_bg)
        # dX / dW pipelining (see module docstring); overlap_dw False: one dX
        # launch then one dW launch per part, on the current stream
        self.overlap_dw = bool(overlap_dw)
        self.bwd_ranges = max(1, int(bwd_ranges))
        self.dw_side_wgs = int(dw_side_wgs)      # workgroups of the overlapped dW launches (0: one per CU)
        self.act_budget = act_budget
        self.max_rays = max_rays                 # explicit cap on rays per part (tests)
        # store-vs-recompute A/B (fine step only): the loss forwards store no
        # dW operand planes; a second forward writes them before the backward
        self.recompute = False
        self._ws = {}                            # device -> grow-only workspace
        self._side = {}                          # device -> side stream
        # called whenever a step starts writing .grad (dp.GradExchange's
        # mark_dirty: a fused zero-grad AdamW step must not mask them)
        self.grad_listeners = []

    # ------------------------------------------------------------ resources
    def _workspace(self, eng, M):
        """Activation workspace for at least M samples (grow-only, per device:
        every call passes its capacity as act_M, so one workspace serves every
        part size)."""
        ws = self._ws.get(eng.device)
        if ws is None or ws["cap"] < M:
            cap = eng.pad(M)
            if ws is not None:
                self._ws.pop(eng.device)
                del ws
            dev = eng.device
            ws = dict(cap=cap, act=eng.new_act(cap),
                      dw=torch.empty(eng.dw_ws_bytes(cap), dtype=torch.uint8, device=dev),
                      dbuf=torch.empty(eng.n_inject, 256, dtype=torch.float32, device=dev),
                      sig=torch.empty(cap, dtype=torch.float32, device=dev),
                      rgb=torch.empty(cap, 3, dtype=torch.float32, device=dev),
                      dsig=torch.empty(cap, dtype=torch.float32, device=dev),
                      drgb=torch.empty(cap, 3, dtype=torch.float32, device=dev))
            self._ws[eng.device] = ws
        return ws

    @staticmethod
    def _zero_pad_rows(ws, layout, ranges):
        """Upstream-gradient rows no loss kernel writes (the padding between
        and after the coarse and fine row ranges) must be 0 for the dX chain.
        They are zeroed when the row layout changes, not every step: nothing
        else writes them."""
        if ws.get("pad_layout") == layout:
            return
        for a, b in ranges:
            if b > a:
                ws["dsig"][a:b].zero_()
                ws["drgb"][a:b].zero_()
        ws["pad_layout"] = layout

    def side_stream(self, device):
        s = self._side.get(device)
        if s is None:
            s = torch.cuda.Stream(device)
            self._side[device] = s
        return s

    def ray_parts(self, eng, R, n_per_ray):
        """Contiguous ray ranges [(a, b)] of whole loss chunks whose training
        workspace (pad(rays x coarse) + rays x fine samples) fits the budget."""
        cap = eng.max_act_samples(self.act_budget)
        per = (cap - 256) // n_per_ray
        if self.max_rays:
            per = min(per, int(self.max_rays))
        per = per // self.chunk * self.chunk
        if per <= 0:
            raise ValueError(f"a loss chunk of {self.chunk} rays x {n_per_ray} samples does not fit the "
                             f"activation budget ({cap} samples): lower the chunk or raise CODENERF_ACT_BUDGET")
        return [(a, min(a + per, R)) for a in range(0, R, per)]

    @staticmethod
    def ensure_grads(tensors):
        for p in tensors:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        return [p.grad for p in tensors]

    def _writing_grads(self):
        for f in self.grad_listeners:
            f()

    # ------------------------------------------------------------ backward
    def _bwd_dw(self, eng, blob, ws, zvec, gtab, M):
        """dX chain + weight gradients over rows [0, M) of the workspace
        (dsig / drgb rows already hold the upstream gradients, padding rows 0),
        pipelined over row ranges on two streams when overlap_dw is set."""
        tm = self.timers
        cap, act = ws["cap"], ws["act"]
        dsig, drgb = ws["dsig"], ws["drgb"]
        Mp = eng.pad(M)
        k = self.bwd_ranges if self.overlap_dw else 1
        k = max(1, min(k, Mp // 256))
        cuts = [(Mp // 256) * i // k * 256 for i in range(k)] + [M]
        ranges = [(cuts[i], cuts[i + 1] - cuts[i]) for i in range(k)]

        # timers: `contended` marks launches that share the chip with a launch
        # on the other stream (the bench reports kernel rooflines from the
        # uncontended ones)
        def bwd(r0, n, ov=False):
            ev = tm.mark("bwd") if tm else None
            eng.mlp_bwd(blob, n, dsig[r0:], drgb[r0:], act, act_M=cap, row0=r0)
            if tm:
                tm.done("bwd", ev, n=n, contended=ov)

        def dw(r0, n, i, nwg, ov=False):
            ev = tm.mark("dw") if tm else None
            eng.mlp_dw(act, n, zvec, gtab, ws["dbuf"], ws["dw"], act_M=cap, row0=r0, db_accum=i > 0, nwg=nwg)
            if tm:
                tm.done("dw", ev, n=n, contended=ov)

        if k == 1:
            bwd(0, M)
            dw(0, M, 0, 0)
            return
        main = torch.cuda.current_stream(eng.device)
        side = self.side_stream(eng.device)
        L = _lib.lib()

        def wait(waiter, signaller):
            # fence-less stream dependency (cn_stream_wait): a torch event's
            # record does a system-scope release -- an L2 write-back of the
            # planes the last kernel wrote, ~15 us of idle GPU per fork / join
            check(L.cn_stream_wait(ctypes.c_void_p(waiter.cuda_stream), ctypes.c_void_p(signaller.cuda_stream)),
                  "cn_stream_wait")

        bwd(*ranges[0])
        for i in range(1, k):
            wait(side, main)
            with torch.cuda.stream(side):
                dw(*ranges[i - 1], i - 1, self.dw_side_wgs, ov=True)
            bwd(*ranges[i], ov=True)
        # the last range's dW runs alone (every CU) on the main stream, right
        # behind its dX chain: the side stream's dW (which shares the partial
        # workspace) finished during that chain, so the join is free, where
        # handing the last dW to the side stream and joining after it added a
        # second cross-stream dependency per step
        wait(main, side)
        dw(*ranges[k - 1], k - 1, 0)

    # ------------------------------------------------------------ steps
    def forward_backward(self, rays_o, viewdirs, z_vals, gt, shape_table, texture_table, obj_idx,
                         reg=True, weight_grads=True):
        """One image: returns (chunk losses [ceil(R/chunk)], rendered rgb [R,3],
        reg loss [1]).  Gradients are accumulated into .grad.  weight_grads
        False (codes-only optimisation, src/optimizer.py): the weight-gradient
        pass is replaced by the bias sums the code gradients need."""
        eng = self.model.engine()
        R = rays_o.shape[0]
        N = z_vals.shape[-1]
        z = z_vals.contiguous().to(eng.device, torch.float32)
        losses, rgbs, regs = [], [], []
        for k, (a, b) in enumerate(self.ray_parts(eng, R, N)):
            zp = z if z.dim() == 1 else z[a:b]
            l, c, r = self._coarse_part(eng, rays_o[a:b], viewdirs[a:b], zp, gt[a:b], shape_table, texture_table,
                                        obj_idx, reg and k == 0, weight_grads)
            losses.append(l)
            rgbs.append(c)
            regs.append(r)
        if len(losses) == 1:
            return losses[0], rgbs[0], regs[0]
        return torch.cat(losses), torch.cat(rgbs), regs[0]

    def _coarse_part(self, eng, rays_o, viewdirs, z, gt, shape_table, texture_table, obj_idx, reg, weight_grads):
        params = self.model.param_list()
        grads = self.ensure_grads(params)
        self.ensure_grads([shape_table, texture_table])
        self._writing_grads()
        R = rays_o.shape[0]
        N = z.shape[-1]
        M = R * N
        z_stride = 0 if z.dim() == 1 else N
        ws = self._workspace(eng, M)
        cap = ws["cap"]
        Mp = eng.pad(M)
        eng.ensure_packed(params, bwd=True)
        s, t = shape_table.detach()[obj_idx], texture_table.detach()[obj_idx]
        blob, zvec = eng.latent_fwd(params, s, t)
        tm = self.timers
        ev = tm.mark("fwd") if tm else None
        sigma, rgb = eng.mlp_fwd(blob, M, rays_o=rays_o, rays_d=viewdirs, z=z, z_stride=z_stride, n_samples=N,
                                 act=ws["act"], act_M=cap, act_row0=0, sigma=ws["sig"][:Mp], rgb=ws["rgb"][:Mp],
                                 codes=not weight_grads)
        if tm:
            tm.done("fwd", ev, n=M)
        dsig, drgb = ws["dsig"], ws["drgb"]
        self._zero_pad_rows(ws, ("coarse", M), [(M, Mp)])
        out_rgb, chunk_loss, _, _ = _eng.render_loss(sigma, rgb, z, R, N, gt, self.chunk, self.white_bg,
                                                     dsig=dsig[:M], drgb=drgb[:M])
        if weight_grads:
            self._bwd_dw(eng, blob, ws, zvec, eng.table(grads), M)
        else:
            ev = tm.mark("bwd") if tm else None
            eng.mlp_bwd(blob, M, dsig, drgb, ws["act"], codes=True, act_M=cap, row0=0)
            if tm:
                tm.done("bwd", ev, n=M)
                ev = tm.mark("dw")
            eng.mlp_dbias(ws["act"], M, ws["dbuf"], ws["dw"], act_M=cap)
            if tm:
                tm.done("dw", ev, n=M)
            grads = ws.setdefault("scratch_grads", [torch.zeros_like(p) for p in params])
        reg_out = torch.empty(1, dtype=torch.float32, device=eng.device)     # written by cn_latent_bwd
        eng.latent_bwd(params, grads, s, t, zvec, ws["dbuf"], shape_table.grad[obj_idx],
                       texture_table.grad[obj_idx], self.reg_coef if reg else 0.0, reg_out)
        return chunk_loss, out_rgb, reg_out

    def forward_backward_fine(self, rays_o, viewdirs, z_c, rand_f, gt, shape_table, texture_table, obj_idx,
                              reg=True, z_f=None):
        """Coarse + fine image step (the BASELINE configs' "64 + 64"; no
        reference counterpart -- NeRF hierarchical sampling through the one
        CodeNeRF MLP, oracle/ref_cpu.py:fine_image_step).  Loss = coarse
        chunk-mean MSE + fine chunk-mean MSE (+ code regulariser once).  The
        coarse pass fills activation rows [0, pad(R*Nc)), the fine pass the
        rows after, so one backward schedule covers both.
        z_f (R, Nf), optional: fine samples to use instead of sample_pdf's
        (tests replaying one sampling under two precisions); rand_f is then
        only read for Nf.
        Returns (coarse chunk losses, fine chunk losses, fine rgb (R,3), reg)."""
        eng = self.model.engine()
        R = rays_o.shape[0]
        Nc, Nf = z_c.shape[-1], rand_f.shape[-1]
        z_c = z_c.contiguous().to(eng.device, torch.float32)
        outs, zfs = [], []
        for k, (a, b) in enumerate(self.ray_parts(eng, R, Nc + Nf)):
            zp = z_c if z_c.dim() == 1 else z_c[a:b]
            outs.append(self._fine_part(eng, rays_o[a:b], viewdirs[a:b], zp, rand_f[a:b], gt[a:b], shape_table,
                                        texture_table, obj_idx, reg and k == 0,
                                        None if z_f is None else z_f[a:b].contiguous()))
            zfs.append(self.last_z_f)
        if len(outs) == 1:
            return outs[0]
        self.last_z_f = torch.cat(zfs)
        return (torch.cat([o[0] for o in outs]), torch.cat([o[1] for o in outs]), torch.cat([o[2] for o in outs]),
                outs[0][3])

    def _fine_part(self, eng, rays_o, viewdirs, z_c, rand_f, gt, shape_table, texture_table, obj_idx, reg,
                   z_f=None):
        params = self.model.param_list()
        grads = self.ensure_grads(params)
        self.ensure_grads([shape_table, texture_table])
        self._writing_grads()
        R = rays_o.shape[0]
        Nc = z_c.shape[-1]
        Nf = rand_f.shape[-1]
        Mc, Mf = R * Nc, R * Nf
        Mc_p = eng.pad(Mc)
        M = Mc_p + Mf
        Mp = eng.pad(M)
        ws = self._workspace(eng, M)
        cap = ws["cap"]
        sig, rgb, dsig, drgb = ws["sig"], ws["rgb"], ws["dsig"], ws["drgb"]
        self._zero_pad_rows(ws, ("fine", Mc, Mf), [(Mc, Mc_p), (Mc_p + Mf, Mp)])
        eng.ensure_packed(params, bwd=True)
        s, t = shape_table.detach()[obj_idx], texture_table.detach()[obj_idx]
        blob, zvec = eng.latent_fwd(params, s, t)
        tm = self.timers
        ev = tm.mark("fwd") if tm else None
        rc = self.recompute
        sig_c, rgb_c = eng.mlp_fwd(blob, Mc, rays_o=rays_o, rays_d=viewdirs, z=z_c,
                                   z_stride=0 if z_c.dim() == 1 else Nc, n_samples=Nc, act=ws["act"], act_M=cap,
                                   act_row0=0, sigma=sig[:Mc_p], rgb=rgb[:Mc_p], codes=rc)
        if tm:
            tm.done("fwd", ev, n=Mc)
        _, loss_c, _, _ = _eng.render_loss(sig_c, rgb_c, z_c, R, Nc, gt, self.chunk, self.white_bg,
                                           dsig=dsig[:Mc], drgb=drgb[:Mc])
        if z_f is None:
            z_f = _eng.sample_pdf(sig_c, z_c, R, Nc, rand_f)
        else:
            z_f = z_f.to(eng.device, torch.float32)
        ev = tm.mark("fwd") if tm else None
        sig_f, rgb_f = eng.mlp_fwd(blob, Mf, rays_o=rays_o, rays_d=viewdirs, z=z_f, z_stride=Nf, n_samples=Nf,
                                   act=ws["act"], act_M=cap, act_row0=Mc_p, sigma=sig[Mc_p:Mp],
                                   rgb=rgb[Mc_p:Mp], codes=rc)
        if tm:
            tm.done("fwd", ev, n=Mf)
        out_f, loss_f = _eng.render_loss_fine(sig_c, rgb_c, z_c, Nc, sig_f, rgb_f, z_f, Nf, R, gt, self.chunk,
                                              dsig[:Mc], drgb[:Mc], dsig[Mc_p:Mc_p + Mf],
                                              drgb[Mc_p:Mc_p + Mf], self.white_bg)
        if rc:
            # recompute A/B (hard part 2): the forward passes above
            # stored only ReLU masks + sigma pre-activations; the planes the dW
            # pass reads are produced here by a second training forward
            if ws.get("dsig_tmp") is None or ws["dsig_tmp"].numel() < cap:   # its (discarded) outputs
                ws["dsig_tmp"] = torch.empty(cap, dtype=torch.float32, device=eng.device)
                ws["drgb_tmp"] = torch.empty(cap, 3, dtype=torch.float32, device=eng.device)
            ev = tm.mark("fwd") if tm else None
            eng.mlp_fwd(blob, Mc, rays_o=rays_o, rays_d=viewdirs, z=z_c, z_stride=0 if z_c.dim() == 1 else Nc,
                        n_samples=Nc, act=ws["act"], act_M=cap, act_row0=0, sigma=ws["dsig_tmp"][:Mc_p],
                        rgb=ws["drgb_tmp"][:Mc_p])
            eng.mlp_fwd(blob, Mf, rays_o=rays_o, rays_d=viewdirs, z=z_f, z_stride=Nf, n_samples=Nf, act=ws["act"],
                        act_M=cap, act_row0=Mc_p, sigma=ws["dsig_tmp"][Mc_p:Mp], rgb=ws["drgb_tmp"][Mc_p:Mp])
            if tm:
                tm.done("fwd", ev)
        self._bwd_dw(eng, blob, ws, zvec, eng.table(grads), M)
        reg_out = torch.empty(1, dtype=torch.float32, device=eng.device)     # written by cn_latent_bwd
        eng.latent_bwd(params, grads, s, t, zvec, ws["dbuf"], shape_table.grad[obj_idx],
                       texture_table.grad[obj_idx], self.reg_coef if reg else 0.0, reg_out)
        self.last_z_f = z_f
        return loss_c, loss_f, out_f, reg_out

    # ------------------------------------------------------------ inference
    @torch.no_grad()
    def render(self, rays_o, viewdirs, z_vals, shape_code, texture_code):
        """Forward only (src/optimizer.py:108-124): -> rgb (R,3), depth (R,).
        No workspace; images beyond CN_MAX_SAMPLES samples go in ray parts."""
        eng = self.model.engine()
        params = self.model.param_list()
        R = rays_o.shape[0]
        N = z_vals.shape[-1]
        z = z_vals.contiguous().to(eng.device, torch.float32)
        eng.ensure_packed(params, bwd=False)
        blob, _ = eng.latent_fwd(params, shape_code.reshape(-1).contiguous(), texture_code.reshape(-1).contiguous())
        per = max(1, (eng.L.cn_max_samples() - 256) // N)
        rgbs, depths = [], []
        for a in range(0, R, per):
            b = min(a + per, R)
            zp = z if z.dim() == 1 else z[a:b]
            sigma, rgb = eng.mlp_fwd(blob, (b - a) * N, rays_o=rays_o[a:b], rays_d=viewdirs[a:b], z=zp,
                                     z_stride=0 if zp.dim() == 1 else N, n_samples=N)
            c, d = _eng.composite_fwd(sigma, rgb, zp, b - a, N, self.white_bg)
            rgbs.append(c)
            depths.append(d)
        if len(rgbs) == 1:
            return rgbs[0], depths[0]
        return torch.cat(rgbs), torch.cat(depths)

    @torch.no_grad()
    def render_sharded(self, rays_o, viewdirs, z_vals, shape_code, texture_code, dist=None, group=None):
        """One image rendered by all ranks (C5 inference):
        rank r renders the contiguous ray block dp.ray_block(R, r) and the
        blocks are all-gathered -> rgb (R,3), depth (R,) on every rank."""
        R = rays_o.shape[0]
        a, b = _dp.ray_block(R, dist, group)
        z = z_vals if z_vals.dim() == 1 else z_vals[a:b]
        if b > a:
            rgb, depth = self.render(rays_o[a:b], viewdirs[a:b], z, shape_code, texture_code)
        else:
            rgb = torch.empty(0, 3, dtype=torch.float32, device=rays_o.device)
            depth = torch.empty(0, dtype=torch.float32, device=rays_o.device)
        return _dp.gather_ray_blocks(rgb, R, dist, group), _dp.gather_ray_blocks(depth, R, dist, group)
