"""GPU checks of the coarse + fine extension (BASELINE configs' "64 + 64").

The reference has no fine pass, so parity is UNPINNED:
these compare the HIP kernels with the CPU restatement in oracle/ref_cpu.py
(sample_pdf, merge_samples, fine_image_step) on identical inputs.

Tolerances: fine z within 1e-5 abs (a float64 cdf rounded once on both
sides; a rare sample whose u sits on a cdf step may move further, so 99.9%
at 1e-5 and all within 1e-3); composite / loss gradients rtol 1e-4 of the
oracle's autograd; the full fp32 step as the coarse-only step test (rgb /
losses rtol 1e-4, parameter gradients rtol 2e-3).
"""
import numpy as np
import pytest
import torch

from golden_util import load, case_params

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("per_ray_z", [False, True])
@pytest.mark.parametrize("Nc,Nf", [(64, 64), (32, 96), (128, 128), (5, 3)])
def test_sample_pdf_matches_oracle(per_ray_z, Nc, Nf):
    from codenerf_amd.engine import sample_pdf
    from oracle import ref_cpu
    g = torch.Generator().manual_seed(Nc * 7 + Nf)
    R = 300
    sig = torch.rand(R, Nc, generator=g) * 8
    sig[:20] = 0.0                                   # empty rays: uniform pdf from the 1e-5 floor
    sig[20:40, Nc // 2] = 1e4                        # opaque walls: degenerate bins
    if per_ray_z:
        z = torch.sort(0.8 + torch.rand(R, Nc, generator=g), -1).values
    else:
        z = torch.linspace(0.8, 1.8, Nc) + torch.rand(Nc, generator=g) / (2 * Nc)
    rnd = torch.rand(R, Nf, generator=g)
    zf = sample_pdf(sig.to(_dev()), z.to(_dev()), R, Nc, rnd.to(_dev())).cpu()
    ref = ref_cpu.sample_pdf(sig, z, rnd)
    d = (zf - ref).abs()
    assert float((d < 1e-5).float().mean()) > 0.999, float(d.max())
    assert float(d.max()) < 1e-3
    assert bool((zf[:, 1:] >= zf[:, :-1]).all()), "fine z must come out sorted"
    zz = z.expand(R, Nc) if z.dim() == 1 else z
    lo = 0.5 * (zz[:, 0] + zz[:, 1])
    hi = 0.5 * (zz[:, -2] + zz[:, -1])
    assert bool((zf >= lo[:, None] - 1e-6).all()) and bool((zf <= hi[:, None] + 1e-6).all())


@pytest.mark.parametrize("Nc,Nf,chunk", [(64, 64, 2048), (32, 32, 100), (96, 160, 77)])
def test_render_loss_fine_matches_oracle(Nc, Nf, chunk):
    from codenerf_amd.engine import render_loss_fine
    from oracle import ref_cpu
    g = torch.Generator().manual_seed(Nc + Nf)
    R = 257
    zc = torch.linspace(0.8, 1.8, Nc)
    zf = torch.sort(0.8 + torch.rand(R, Nf, generator=g), -1).values
    zf[0, :4] = zc[3]                                # ties: coarse first
    sc = (torch.rand(R, Nc, generator=g) * 6).requires_grad_()
    rc = torch.randn(R, Nc, 3, generator=g).requires_grad_()
    sf = (torch.rand(R, Nf, generator=g) * 6).requires_grad_()
    rf = torch.randn(R, Nf, 3, generator=g).requires_grad_()
    gt = torch.rand(R, 3, generator=g)
    # an already-present coarse gradient, small so (dsc0 + grad) - dsc0 keeps grad's bits
    dsc0 = torch.randn(R * Nc, generator=g) * 1e-9
    drc0 = torch.randn(R * Nc, 3, generator=g) * 1e-9
    dv = _dev()
    dsc, drc = dsc0.clone().to(dv), drc0.clone().to(dv)
    dsf = torch.empty(R * Nf, device=dv)
    drf = torch.empty(R * Nf, 3, device=dv)
    rgb, losses = render_loss_fine(sc.detach().to(dv), rc.detach().to(dv), zc.to(dv), Nc, sf.detach().to(dv),
                                   rf.detach().to(dv), zf.to(dv), Nf, R, gt.to(dv), chunk, dsc, drc, dsf, drf)
    # oracle: chunk-mean MSE over the merged composite, summed over chunks
    z_m, s_m, r_m = ref_cpu.merge_samples(zc, zf, (sc, sf), (rc, rf))
    out, _ = ref_cpu.volume_rendering(s_m, r_m, z_m)
    tot, ref_losses = 0.0, []
    for a in range(0, R, chunk):
        l2 = torch.mean((out[a:a + chunk] - gt[a:a + chunk]) ** 2)
        ref_losses.append(l2.item())
        tot = tot + l2
    tot.backward()
    np.testing.assert_allclose(rgb.cpu().numpy(), out.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(losses.cpu().numpy(), np.array(ref_losses), rtol=1e-5)
    sc_g = (dsc.cpu() - dsc0).reshape(R, Nc)
    np.testing.assert_allclose(sc_g.numpy(), sc.grad.numpy(), rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose((drc.cpu() - drc0).reshape(R, Nc, 3).numpy(), rc.grad.numpy(), rtol=1e-4,
                               atol=1e-8)
    np.testing.assert_allclose(dsf.cpu().reshape(R, Nf).numpy(), sf.grad.numpy(), rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(drf.cpu().reshape(R, Nf, 3).numpy(), rf.grad.numpy(), rtol=1e-4, atol=1e-8)


def _fine_step(g, precision, Nf, rnd, overlap_dw=True):
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.render import ImageStep
    m = CodeNeRF(3, 1, precision=precision)
    m.load_state_dict({k: torch.tensor(v) for k, v in case_params(g).items()})
    m = m.to(_dev())
    st = torch.nn.Parameter(torch.tensor(g["shape_table"], device=_dev()))
    tt = torch.nn.Parameter(torch.tensor(g["texture_table"], device=_dev()))
    step = ImageStep(m, chunk=int(g["chunk"]), reg_coef=1e-4, overlap_dw=overlap_dw)
    ro = torch.tensor(g["rays_o"], device=_dev())
    vd = torch.tensor(g["viewdir"], device=_dev())
    z = torch.tensor(g["z_vals"], device=_dev())
    gt = torch.tensor(g["gt"], device=_dev())
    lc, lf, rgb, reg = step.forward_backward_fine(ro, vd, z, rnd.to(_dev()), gt, st, tt, int(g["obj_idx"]))
    torch.cuda.synchronize()
    return m, st, tt, lc, lf, rgb, step.last_z_f


@pytest.mark.parametrize("case,Nf,nrays", [("n64_16x16", 64, 0), ("c1_32x32_n32", 32, 0), ("ragged_48x48_n16", 40, 0),
                                           ("chunks_64x64_n16", 16, 0), ("n64_16x16", 64, 1), ("c1_32x32_n32", 32, 3)])
def test_fine_train_step_fp32_matches_oracle(case, Nf, nrays):
    """nrays > 0: the first rays of the case only (one ray: 64 + 64 samples in
    one partial tile, a single partial loss chunk)."""
    from oracle import ref_cpu
    g = load(case)
    if nrays:
        g = dict(g)
        for k in ("rays_o", "viewdir", "gt"):
            g[k] = g[k][:nrays]
    R = g["rays_o"].shape[0]
    rnd = torch.rand(R, Nf, generator=torch.Generator().manual_seed(5))
    m, st, tt, lc, lf, rgb, zf = _fine_step(g, "fp32", Nf, rnd)
    p = ref_cpu.param_tensors(case_params(g))
    st_r = torch.tensor(g["shape_table"], requires_grad=True)
    tt_r = torch.tensor(g["texture_table"], requires_grad=True)
    ro, vd, z = torch.tensor(g["rays_o"]), torch.tensor(g["viewdir"]), torch.tensor(g["z_vals"])
    # the oracle's own fine z from its coarse densities agrees with the GPU's
    with torch.no_grad():
        xyz = ro[:, None, :] + vd[:, None, :] * z[:, None]
        oi = int(g["obj_idx"])
        sig_c, _ = ref_cpu.codenerf_forward(p, xyz, vd[:, None, :].expand(-1, z.numel(), -1),
                                            st_r[oi][None], tt_r[oi][None])
        zf_ref = ref_cpu.sample_pdf(sig_c[..., 0], z, rnd)
    assert float((zf.cpu() - zf_ref).abs().max()) < 1e-4
    # the step itself, replayed on the GPU's fine z
    lc_r, lf_r, rgb_r = ref_cpu.fine_image_step(p, st_r, tt_r, oi, ro, vd, z, zf.cpu(), torch.tensor(g["gt"]),
                                                chunk=int(g["chunk"]))
    np.testing.assert_allclose(rgb.cpu().numpy(), rgb_r.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(lc.cpu().numpy(), np.array(lc_r), rtol=1e-4)
    np.testing.assert_allclose(lf.cpu().numpy(), np.array(lf_r), rtol=1e-4)
    for k, prm in m.named_parameters():
        a, b = prm.grad.cpu().numpy(), p[k].grad.numpy()
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-6 * max(1.0, np.abs(b).max()), err_msg=k)
    sg = st.grad.cpu().numpy()
    np.testing.assert_allclose(sg, st_r.grad.numpy(), rtol=2e-3, atol=2e-6 * max(1.0, np.abs(sg).max()))
    tg = tt.grad.cpu().numpy()
    np.testing.assert_allclose(tg, tt_r.grad.numpy(), rtol=2e-3, atol=2e-6 * max(1.0, np.abs(tg).max()))


def test_fine_train_step_bf16_close_to_fp32():
    g = load("n64_16x16")
    R = g["rays_o"].shape[0]
    rnd = torch.rand(R, 64, generator=torch.Generator().manual_seed(6))
    m32, st32, _, lc32, lf32, rgb32, zf32 = _fine_step(g, "fp32", 64, rnd)
    m16, st16, _, lc16, lf16, rgb16, zf16 = _fine_step(g, "bf16", 64, rnd)
    assert np.abs(rgb16.cpu().numpy() - rgb32.cpu().numpy()).max() < 3e-2
    np.testing.assert_allclose(lf16.cpu().numpy(), lf32.cpu().numpy(), rtol=3e-2)
    for (k, a), (_, b) in zip(m16.named_parameters(), m32.named_parameters()):
        if b.grad.abs().max() > 0:
            a_, b_ = a.grad.reshape(-1).double(), b.grad.reshape(-1).double()
            assert float(a_ @ b_ / (a_.norm() * b_.norm())) > 0.98, k


@pytest.mark.parametrize("precision,case,Nf", [("fp32", "ragged_48x48_n16", 40), ("bf16", "n64_16x16", 64),
                                               ("bf16", "chunks_64x64_n16", 16)])
def test_overlapped_bwd_dw_matches_single_pass(precision, case, Nf):
    """ImageStep(overlap_dw=True): dX chain + dW split at the coarse / fine
    row boundary on two streams (cn_mlp_bwd_rows / cn_mlp_dw_rows) gives the
    gradients of the one-launch path (same sums, fp32 partial order aside)."""
    g = load(case)
    R = g["rays_o"].shape[0]
    rnd = torch.rand(R, Nf, generator=torch.Generator().manual_seed(8))
    a = _fine_step(g, precision, Nf, rnd, overlap_dw=True)
    b = _fine_step(g, precision, Nf, rnd, overlap_dw=False)
    np.testing.assert_array_equal(a[4].cpu().numpy(), b[4].cpu().numpy())      # fine losses
    for (k, pa), (_, pb) in zip(a[0].named_parameters(), b[0].named_parameters()):
        x, y = pa.grad.cpu().numpy(), pb.grad.cpu().numpy()
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5 * max(1e-30, np.abs(y).max()), err_msg=k)
    for i in (1, 2):
        x, y = a[i].grad.cpu().numpy(), b[i].grad.cpu().numpy()
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5 * max(1e-30, np.abs(y).max()))


def test_recompute_schedule_matches_store_schedule():
    """The store-vs-recompute A/B (ImageStep.recompute: loss forwards keep only
    masks, a second forward writes the dW operand planes) computes the same
    step bit for bit -- it differs only in time."""
    g = load("n64_16x16")
    R = g["rays_o"].shape[0]
    rnd = torch.rand(R, 64, generator=torch.Generator().manual_seed(12))
    outs = []
    for rc in (False, True):
        from codenerf_amd.model import CodeNeRF
        from codenerf_amd.render import ImageStep
        m = CodeNeRF(3, 1, precision="bf16")
        m.load_state_dict({k: torch.tensor(v) for k, v in case_params(g).items()})
        m = m.to(_dev())
        st = torch.nn.Parameter(torch.tensor(g["shape_table"], device=_dev()))
        tt = torch.nn.Parameter(torch.tensor(g["texture_table"], device=_dev()))
        step = ImageStep(m, chunk=int(g["chunk"]), reg_coef=1e-4)
        step.recompute = rc
        lc, lf, rgb, _ = step.forward_backward_fine(torch.tensor(g["rays_o"], device=_dev()),
                                                    torch.tensor(g["viewdir"], device=_dev()),
                                                    torch.tensor(g["z_vals"], device=_dev()), rnd.to(_dev()),
                                                    torch.tensor(g["gt"], device=_dev()), st, tt, int(g["obj_idx"]))
        torch.cuda.synchronize()
        outs.append([lf.cpu(), rgb.cpu()] + [p.grad.cpu() for p in m.parameters()] + [st.grad.cpu()])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
