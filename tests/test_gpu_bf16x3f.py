"""GPU: the bf16x3f plan (CN_BF16X3F) -- the bf16x3 forward chains with the
bf16 backward.

What it must be, and what is checked here:
  * its forward IS the bf16x3 forward: rendered rgb, chunk losses and every
    plane the bf16 backward reads (PE, dir, Y, ReLU masks, sigma
    pre-activations) bit-identical to a bf16x3 plan's on the same inputs (the
    bf16x3 plan stores the X lo planes after those, at the offsets beyond
    the bf16 layout);
  * rendered rgb within the north-star bar (1e-4 relative) of the reference
    goldens and of the fp32 oracle at C2 size (test_c2_fp32_class_rgb in
    test_gpu_configs.py);
  * gradients at the bf16 backward's precision: rel-L2 vs the float64 replay
    <= 2e-2 (the bf16 bar), and close to the oracle run at the same operand
    precision (ref_cpu.bf16_operands(ops=OPS_BF16X3F)).
"""
import numpy as np
import pytest
import torch

from golden_util import TRAIN_CASES, case_params, load, oracle64_image_step

pytestmark = pytest.mark.gpu

RGB_REL = 1e-4          # north-star rgb bar (relative to the reference's rgb)
GRAD_REL = 2e-2         # the bf16 backward's bar vs float64 (test_gpu_bf16x3.py X3_GRAD_REL)


def _dev():
    return torch.device("cuda", 0)


def _step(g, precision):
    from codenerf_amd.model import CodeNeRF
    from codenerf_amd.render import ImageStep
    m = CodeNeRF(3, 1, precision=precision)
    m.load_state_dict({k: torch.tensor(v) for k, v in case_params(g).items()})
    m = m.to(_dev())
    st = torch.nn.Parameter(torch.tensor(g["shape_table"], device=_dev()))
    tt = torch.nn.Parameter(torch.tensor(g["texture_table"], device=_dev()))
    step = ImageStep(m, chunk=int(g["chunk"]), reg_coef=1e-4)
    t = lambda k: torch.tensor(g[k], device=_dev())
    losses, rgb, _ = step.forward_backward(t("rays_o"), t("viewdir"), t("z_vals"), t("gt"), st, tt, int(g["obj_idx"]))
    torch.cuda.synchronize()
    return m, st, tt, losses.cpu().numpy(), rgb.cpu().numpy()


def _oracle(g, ops):
    from oracle import ref_cpu
    p = ref_cpu.param_tensors(case_params(g))
    st = torch.tensor(g["shape_table"], requires_grad=True)
    tt = torch.tensor(g["texture_table"], requires_grad=True)
    f = lambda k: torch.tensor(g[k])
    with ref_cpu.bf16_operands(ops=ops):
        losses, rgb = ref_cpu.image_step(p, st, tt, int(g["obj_idx"]), f("rays_o"), f("viewdir"), f("z_vals"),
                                         f("gt"), chunk=int(g["chunk"]))
    return p, st, tt, np.array(losses), rgb.numpy()


def _rel(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


@pytest.mark.parametrize("case", TRAIN_CASES)
def test_bf16x3f_train_step_vs_reference(case):
    from oracle import ref_cpu
    g = load(case)
    mf, stf, ttf, lf, rgbf = _step(g, "bf16x3f")
    _, _, _, l3, rgb3 = _step(g, "bf16x3")
    m16, _, _, _, _ = _step(g, "bf16")
    # the forward is the bf16x3 forward, bit for bit
    assert np.array_equal(rgbf, rgb3) and np.array_equal(lf, l3)
    ref = np.asarray(g["rgb"], np.float64)
    rel = float((np.abs(rgbf - ref) / np.maximum(np.abs(ref), 1e-2)).max())
    r64 = oracle64_image_step(g)
    p_x, st_x, tt_x, l_x, rgb_x = _oracle(g, ref_cpu.OPS_BF16X3F)
    gerr = {k: _rel(p.grad.cpu().numpy(), r64["params"][k].grad.numpy()) for k, p in mf.named_parameters()}
    gerr16 = {k: _rel(p.grad.cpu().numpy(), r64["params"][k].grad.numpy()) for k, p in m16.named_parameters()}
    gerr_x = {k: _rel(p.grad.cpu().numpy(), p_x[k].grad.numpy()) for k, p in mf.named_parameters()}
    print(f"\n{case}: bf16x3f rgb max rel vs golden {rel:.2e} (max|d| {np.abs(rgbf - ref).max():.2e}); "
          f"grad rel-L2 vs f64 worst {max(gerr.values()):.2e} (bf16 plan {max(gerr16.values()):.2e}); "
          f"vs its same-precision oracle worst {max(gerr_x.values()):.2e}")
    assert rel <= RGB_REL
    np.testing.assert_allclose(lf, g["chunk_losses"], rtol=2e-4)
    assert max(gerr.values()) <= GRAD_REL, gerr
    # the same-precision oracle rounds the same operands but sums in another
    # order (and forms encoding_shape's gradient per layer, not by the fold)
    assert max(gerr_x.values()) <= 1e-2, gerr_x
    for tab, refg in ((stf, r64["shape_table"]), (ttf, r64["texture_table"])):
        assert _rel(tab.grad.cpu().numpy(), refg.grad.numpy()) <= GRAD_REL


def test_bf16x3f_planes_equal_bf16x3_hi_planes():
    """C2-size ragged batch: the bf16x3f training forward stores exactly the
    bf16x3 plan's hi planes, masks and sigma pre-activations (its workspace
    is the bf16x3 workspace without the lo planes appended after them), and
    the bf16 backward then runs on them (finite, non-zero gradients)."""
    from codenerf_amd.model import CodeNeRF
    torch.manual_seed(0)
    mf = CodeNeRF(3, 1, precision="bf16x3f").to(_dev())
    m3 = CodeNeRF(3, 1, precision="bf16x3").to(_dev())
    m3.load_state_dict(mf.state_dict())
    R, N = 128 * 128 - 37, 64
    ro = torch.zeros(R, 3, device=_dev()) + torch.tensor([0.0, 0.4, 1.2], device=_dev())
    vd = torch.nn.functional.normalize(torch.randn(R, 3, device=_dev()) * 0.2
                                       + torch.tensor([0., -0.3, -1.], device=_dev()), dim=-1)
    z = torch.linspace(0.8, 1.8, N, device=_dev())
    s = torch.randn(256, device=_dev()) / 11.3
    t = torch.randn(256, device=_dev()) / 11.3
    M = R * N
    outs = {}
    for name, m in (("x3f", mf), ("x3", m3)):
        eng = m.engine()
        params = m.param_list()
        eng.ensure_packed(params)
        blob, zvec = eng.latent_fwd(params, s, t)
        act = torch.zeros(eng.act_bytes(M), dtype=torch.uint8, device=_dev())
        sig, rgb = eng.mlp_fwd(blob, M, rays_o=ro, rays_d=vd, z=z, n_samples=N, act=act)
        outs[name] = (eng, params, blob, zvec, act, sig[:M].clone(), rgb[:M].clone())
    torch.cuda.synchronize()
    ef, af, a3 = outs["x3f"][0], outs["x3f"][4], outs["x3"][4]
    assert a3.numel() > af.numel()
    assert torch.equal(outs["x3f"][5], outs["x3"][5]) and torch.equal(outs["x3f"][6], outs["x3"][6])
    assert torch.equal(af, a3[:af.numel()]), "bf16x3f planes differ from the bf16x3 hi planes"
    eng, params, blob, zvec, act = outs["x3f"][:5]
    Mp = eng.pad(M)
    dsig = torch.zeros(Mp, device=_dev())
    drgb = torch.zeros(Mp, 3, device=_dev())
    dsig[:M] = torch.randn(M, device=_dev()) * 1e-3
    drgb[:M] = torch.randn(M, 3, device=_dev()) * 1e-3
    eng.mlp_bwd(blob, M, dsig, drgb, act)
    grads = [torch.zeros_like(p) for p in params]
    dbuf = torch.zeros(eng.n_inject, 256, device=_dev())
    eng.mlp_dw(act, M, zvec, grads, dbuf)
    torch.cuda.synchronize()
    assert all(torch.isfinite(gr).all() for gr in grads)
    assert sum(float(gr.abs().sum()) for gr in grads) > 0


def test_bf16x3f_module_api_and_default_net():
    """The per-sample module API (CodeNeRF.forward + autograd) on the
    reference's default net (2 shape blocks): forward within RGB_REL of the
    fp32 oracle, gradients within GRAD_REL of the float64 oracle."""
    from codenerf_amd.model import CodeNeRF
    from oracle import ref_cpu
    from oracle.params import make_codes, make_params
    g = load("n64_16x16")
    params = make_params(44, shape_blocks=2)
    s0, t0 = make_codes(44, 3)
    m = CodeNeRF(2, 1, precision="bf16x3f")
    m.load_state_dict({k: torch.tensor(v) for k, v in params.items()})
    m = m.to(_dev())
    ro, vd, z = torch.tensor(g["rays_o"]), torch.tensor(g["viewdir"]), torch.tensor(g["z_vals"])
    xyz = (ro[:, None, :] + vd[:, None, :] * z[:, None]).to(_dev())
    vrep = vd[:, None, :].expand(-1, z.numel(), -1).contiguous().to(_dev())
    s = torch.tensor(s0[1:2], device=_dev())
    t = torch.tensor(t0[1:2], device=_dev())
    sig, rgbs = m(xyz, vrep, s, t)
    w = torch.randn_like(rgbs)
    ((rgbs * w).sum() + sig.sum()).backward()
    p64 = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in params.items()}
    sr, rr = ref_cpu.codenerf_forward(p64, xyz.cpu().double(), vrep.cpu().double(), torch.tensor(s0[1:2]).double(),
                                      torch.tensor(t0[1:2]).double(), shape_blocks=2)
    ((rr * w.cpu().double()).sum() + sr.sum()).backward()
    er = float((rgbs.detach().cpu().double() - rr.detach()).abs().max() / rr.detach().abs().max())
    es = float((sig.detach().cpu().double() - sr.detach()).abs().max() / sr.detach().abs().max())
    gerr = {k: _rel(p.grad.cpu().numpy(), p64[k].grad.numpy()) for k, p in m.named_parameters()}
    print(f"\nbf16x3f module (2 shape blocks): rgb rel {er:.2e}, sigma rel {es:.2e}, "
          f"grad rel-L2 worst {max(gerr.values()):.2e}")
    assert er <= RGB_REL and es <= RGB_REL
    assert max(gerr.values()) <= GRAD_REL, gerr
