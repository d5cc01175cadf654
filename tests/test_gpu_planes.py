"""GPU: the activation planes the bf16 chain kernels store, element by element.

Targets the gfx950 store hazard the chain epilogues work around (chain.hip
plane_store_pair: a buffer store whose data comes straight from
v_permlane32_swap read its first data dword after the next VALU had
rewritten it, so mask bits appeared in stored values).  The workaround
depends on wait states, so a compiler scheduling change could reintroduce
it silently; this test decodes every element of the stored planes (layout:
cn_layout.h slab_off, restated below) at several sample counts, ragged tails
included, and compares them with a torch emulation of the bf16 chain
(bf16 operands, fp32 accumulation, bf16 storage):

  * PE plane (64 slot columns)  vs bf16(PE(x))            -- forward prologue
  * Y planes of layers 0, 2, 5, 7 (enc_xyz, shape_2, enc_viewdir, rgb.0); the
    encoding_shape planes (layer 4) are not stored (reported absent)
  * dA plane of rgb.0 (first backward epilogue) and of the PE layer (last)

Bar: >= 99% of elements within 1 bf16 ulp (accumulation order and the
rounding boundary), every element within 4 ulps + 1e-3 -- a corrupted dword
is off by orders of magnitude.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle.params import make_codes, make_params

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _pe_slot_feature(h, s):
    """cn_layout.h pe_slot_feature."""
    if s == 0:
        return 0 if h == 0 else 2
    if s == 1:
        return 1 if h == 0 else -1
    k = (s - 2) >> 1
    p = 15 * h + k
    return 3 + p if (s & 1) == 0 else 33 + p


def _decode(buf, off, F, M):
    """bf16 plane of width F at byte offset ``off`` -> (M, F) float32
    (cn_layout.h: slab of 32 samples = F/32 tiles of two 1 KiB pair blocks;
    sample s, features 16gp + 4hh .. +3 and 16gp + 8 + 4hh .. +3 at position
    32hh + ((s + 8gp + 4hh) & 31), in its first and second 8 bytes)."""
    m = np.arange(M)[:, None]
    f = np.arange(F)[None, :]
    s = m & 31
    gp, gg, hh = (f >> 4) & 1, (f >> 3) & 1, (f >> 2) & 1
    pos = 32 * hh + ((s + 8 * gp + 4 * hh) & 31)
    byte = (m >> 5) * F * 64 + (f >> 5) * 2048 + gp * 1024 + pos * 16 + gg * 8 + (f & 3) * 2
    raw = buf[off:].view(torch.int16).cpu().numpy()
    vals = raw[(byte // 2).reshape(-1)].reshape(M, F).astype(np.int32) << 16
    return torch.from_numpy(vals.view(np.float32).copy())


def _check(name, got, want):
    ulp = torch.clamp(want.abs(), min=2.0 ** -126) * 2.0 ** -7      # one bf16 ulp (upper bound)
    d = (got - want).abs()
    close = (d <= ulp + 1e-6).float().mean().item()
    worst = (d - 4 * ulp - 1e-3).max().item()
    assert close >= 0.99 and worst <= 0, (name, close, float(d.max()))


def _pe(x, L):
    ys = [x * (2.0 ** i) for i in range(L)]
    y = torch.cat(ys, -1)
    return torch.cat([x, torch.sin(y), torch.cos(y)], -1)


@pytest.mark.parametrize("M", [256, 4096 + 37, 32768 + 160])
def test_bf16_planes_match_emulation(M):
    from codenerf_amd.model import CodeNeRF
    dev = torch.device("cuda", 0)
    params = make_params(81)
    m = CodeNeRF(3, 1, precision="bf16")
    m.load_state_dict({k: torch.tensor(v) for k, v in params.items()})
    m = m.to(dev)
    eng = m.engine()
    P = {k: torch.tensor(v) for k, v in params.items()}
    g = torch.Generator().manual_seed(M)
    xyz = torch.rand(M, 3, generator=g) * 2 - 1
    vd = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
    s0, t0 = (torch.tensor(c[0]) for c in make_codes(81, 1))
    plist = m.param_list()
    eng.ensure_packed(plist)
    blob, zvec = eng.latent_fwd(plist, s0.to(dev), t0.to(dev))
    act = eng.new_act(M)
    act.zero_()
    eng.mlp_fwd(blob, M, xyz=xyz.to(dev), viewdir=vd.to(dev), act=act)
    drgb = torch.randn(M, 3, generator=g) * 1e-3
    dsig = torch.zeros(M)
    eng.mlp_bwd(blob, M, dsig.to(dev), drgb.to(dev), act)
    torch.cuda.synchronize()

    def plane(kind, idx):
        w = ctypes.c_int()
        off = eng.L.cn_act_plane(eng._plan, M, kind, idx, ctypes.byref(w))
        assert off >= 0
        return off, w.value

    # PE plane: slot columns -> reference features
    off, F = plane(2, 0)
    pe_ref = _bf(_pe(xyz, 10))
    got = _decode(act, off, F, M)
    cols = [(c, _pe_slot_feature((c >> 2) & 1, 4 * (c >> 3) + (c & 3))) for c in range(F)]
    keep = [(c, f) for c, f in cols if f >= 0]
    _check("pe", got[:, [c for c, _ in keep]], pe_ref[:, [f for _, f in keep]])

    # forward emulation: bf16 operands, fp32 accumulation, bf16 storage
    def lin(name, x):
        return _bf(x) @ _bf(P[name + ".weight"]).t()

    def zinj(kind, j, code):
        return torch.relu(code[None] @ P[f"{kind}_latent_layer_{j}.0.weight"].t() + P[f"{kind}_latent_layer_{j}.0.bias"])

    ys = {}
    y = torch.relu(lin("encoding_xyz.0", pe_ref) + P["encoding_xyz.0.bias"])
    ys[0] = _bf(y)
    for j in range(1, 4):
        W = P[f"shape_layer_{j}.0.weight"]
        bias = P[f"shape_layer_{j}.0.bias"] + zinj("shape", j, s0) @ W.t()
        y = torch.relu(lin(f"shape_layer_{j}.0", ys[j - 1]) + bias)
        ys[j] = _bf(y)
    ys[4] = _bf(lin("encoding_shape", ys[3]) + P["encoding_shape.bias"])
    vpe = _bf(_pe(vd, 4))
    y = torch.relu(_bf(torch.cat([ys[4], vpe], -1)) @ _bf(P["encoding_viewdir.0.weight"]).t()
                   + P["encoding_viewdir.0.bias"])
    ys[5] = _bf(y)
    W = P["texture_layer_1.0.weight"]
    y = torch.relu(lin("texture_layer_1.0", ys[5]) + P["texture_layer_1.0.bias"] + zinj("texture", 1, t0) @ W.t())
    ys[6] = _bf(y)
    pre7 = lin("rgb.0", ys[6]) + P["rgb.0.bias"]
    ys[7] = _bf(torch.relu(pre7))
    for i in (0, 2, 5, 7):
        off, F = plane(0, i)
        _check(f"Y{i}", _decode(act, off, F, M), ys[i])
    for kind in (0, 1):      # encoding_shape's Y / dA: folded, never written
        w = ctypes.c_int()
        assert eng.L.cn_act_plane(eng._plan, M, kind, 4, ctypes.byref(w)) == -1 and w.value == 0

    # first backward epilogue: dA(rgb.0) = mask * (W_rgb2^T drgb)
    off, F = plane(1, 7)
    da7 = _bf((_bf(drgb) @ _bf(P["rgb.2.weight"])) * (pre7 > 0))
    _check("dA7", _decode(act, off, F, M), da7)
    # last backward epilogue: dA of the PE layer; its input is the stored dA
    # of layer 1, so it is checked against the kernel's own upstream plane
    off1, F1 = plane(1, 1)
    da1 = _decode(act, off1, F1, M)
    pre0 = lin("encoding_xyz.0", pe_ref) + P["encoding_xyz.0.bias"]
    da0 = _bf((da1 @ _bf(P["shape_layer_1.0.weight"])) * (pre0 > 0))
    off0, F0 = plane(1, 0)
    _check("dA0", _decode(act, off0, F0, M), da0)


@pytest.mark.parametrize("M", [4096 + 37])
def test_bf16x3_lo_planes_carry_the_residual(M):
    """bf16x3 training forward: every X operand of dW is stored as a hi plane
    and a lo plane (rn(x - rn(x)), CN_PLANE_YLO / CN_PLANE_PELO) so the
    weight gradients multiply ~16 significant bits.  hi + lo of the PE plane
    and of Y planes 0, 2, 5, 7 against an fp32 forward (the bf16x3 chains
    track fp32 to ~2^-16 per layer); a lo plane corrupted by the store hazard
    or mis-addressed would be off by orders of magnitude."""
    from codenerf_amd.model import CodeNeRF
    dev = torch.device("cuda", 0)
    params = make_params(82)
    m = CodeNeRF(3, 1, precision="bf16x3")
    m.load_state_dict({k: torch.tensor(v) for k, v in params.items()})
    m = m.to(dev)
    eng = m.engine()
    P = {k: torch.tensor(v, dtype=torch.float64) for k, v in params.items()}
    g = torch.Generator().manual_seed(M)
    xyz = torch.rand(M, 3, generator=g) * 2 - 1
    vd = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
    s0, t0 = (torch.tensor(c[0]) for c in make_codes(82, 1))
    plist = m.param_list()
    eng.ensure_packed(plist)
    blob, _ = eng.latent_fwd(plist, s0.to(dev), t0.to(dev))
    act = eng.new_act(M)
    act.zero_()
    eng.mlp_fwd(blob, M, xyz=xyz.to(dev), viewdir=vd.to(dev), act=act)
    torch.cuda.synchronize()

    def plane(kind, idx):
        w = ctypes.c_int()
        off = eng.L.cn_act_plane(eng._plan, M, kind, idx, ctypes.byref(w))
        assert off >= 0, (kind, idx)
        return off, w.value

    def both(kind_hi, kind_lo, idx):
        off, F = plane(kind_hi, idx)
        offl, Fl = plane(kind_lo, idx)
        assert Fl == F
        hi, lo = _decode(act, off, F, M), _decode(act, offl, F, M)
        # the lo part is below half a bf16 ulp of the hi part
        assert bool((lo.abs() <= hi.abs() * 2.0 ** -8 + 1e-30).all())
        return hi.double() + lo.double()

    def check(name, got, want):
        scale = want.abs().max().item()
        d = (got - want).abs()
        close = (d <= 2e-4 * want.abs() + 1e-5 * scale).double().mean().item()
        assert close >= 0.99 and d.max().item() <= 1e-3 * scale, (name, close, d.max().item(), scale)

    x64, v64 = xyz.double(), vd.double()
    pe = _pe(x64, 10)
    got = both(2, 6, 0)
    cols = [(c, _pe_slot_feature((c >> 2) & 1, 4 * (c >> 3) + (c & 3))) for c in range(64)]
    keep = [(c, f) for c, f in cols if f >= 0]
    check("pe hi+lo", got[:, [c for c, _ in keep]], pe[:, [f for _, f in keep]])
    d = (got[:, [c for c, _ in keep]] - pe[:, [f for _, f in keep]]).abs()
    assert d.max().item() <= 2.0 ** -15, d.max().item()      # 16+ significant bits of a |x| <= 2 feature

    def lin(name, x):
        return x @ P[name + ".weight"].t() + P[name + ".bias"]

    def zinj(kind, j, code):
        return torch.relu(code.double()[None] @ P[f"{kind}_latent_layer_{j}.0.weight"].t()
                          + P[f"{kind}_latent_layer_{j}.0.bias"])

    ys = {0: torch.relu(lin("encoding_xyz.0", pe))}
    for j in range(1, 4):
        ys[j] = torch.relu(lin(f"shape_layer_{j}.0", ys[j - 1] + zinj("shape", j, s0)))
    ys[4] = lin("encoding_shape", ys[3])
    ys[5] = torch.relu(lin("encoding_viewdir.0", torch.cat([ys[4], _pe(v64, 4)], -1)))
    ys[6] = torch.relu(lin("texture_layer_1.0", ys[5] + zinj("texture", 1, t0)))
    ys[7] = torch.relu(lin("rgb.0", ys[6]))
    for i in (0, 2, 5, 7):
        check(f"Y{i} hi+lo", both(0, 5, i), ys[i])
    w = ctypes.c_int()
    assert eng.L.cn_act_plane(eng._plan, M, 5, 4, ctypes.byref(w)) == -1      # encoding_shape: folded
