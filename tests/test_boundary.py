"""CPU-tier checks of the drop-in boundary: the C-ABI library loads and exports
exactly what include/codenerf.h declares; the host package imports; product
calls fail loudly without a HIP device (no CPU fallback)."""
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "codenerf.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cn_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_binding():
    import codenerf_amd._lib as L
    assert sorted(L.EXPORTED) == declared_symbols()


def test_library_loads_and_exports_every_symbol():
    import codenerf_amd._lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("library not built")
    lib = L.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.cn_abi_version() == L.ABI_VERSION


def test_no_cpu_fallback():
    import codenerf_amd._lib as L
    from codenerf_amd.model import CodeNeRF
    if torch.cuda.is_available():
        pytest.skip("device present")
    m = CodeNeRF(3, 1)
    x = torch.zeros(4, 8, 3)
    with pytest.raises(RuntimeError):
        m(x, x, torch.zeros(1, 256), torch.zeros(1, 256))
    with pytest.raises(L.HipUnavailable):
        L.lib()


def test_state_dict_names_match_reference():
    from codenerf_amd.model import CodeNeRF
    from oracle.params import param_specs
    m = CodeNeRF(3, 1)
    sd = m.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, tuple(s)) for k, s in param_specs(3, 1)]


def _plan(lib, precision=1):
    import ctypes
    h = ctypes.c_void_p()
    assert lib.cn_plan_create(3, 1, 256, 10, 4, 256, precision, ctypes.byref(h)) == 0, lib.cn_last_error()
    return h


def test_plan_and_size_queries_need_no_device():
    import codenerf_amd._lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("library not built")
    lib = L.load_library()
    for prec in (0, 1):
        h = _plan(lib, prec)
        assert lib.cn_plan_num_params(h) == 28
        assert lib.cn_pad_samples(h, 1) == 256
        assert lib.cn_pad_samples(h, lib.cn_max_samples() + 1) == -1
        per = lib.cn_act_bytes_per_sample(h)
        # bf16: ~8.2 KB of planes per training sample, fp32 about twice that
        assert (7_000 if prec else 14_000) < per < (9_000 if prec else 18_000)
        assert lib.cn_act_bytes(h, 1 << 20) == per << 20
        lib.cn_plan_destroy(h)


def test_bf16x3f_plan_composes_the_bf16x3_forward_and_the_bf16_backward():
    """CN_BF16X3F: the forward pack of the bf16x3 plan (W_hi + W_lo
    fragments), the backward pack and the workspace of the bf16 plan (its
    training forward stores the bf16 planes only); bf16x3's workspace is the
    same layout with the X lo planes appended."""
    import codenerf_amd._lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("library not built")
    lib = L.load_library()
    h16, h3, h3f = _plan(lib, L.CN_BF16), _plan(lib, L.CN_BF16X3), _plan(lib, L.CN_BF16X3F)
    assert lib.cn_packed_bytes(h3f, 0) == lib.cn_packed_bytes(h3, 0) > lib.cn_packed_bytes(h16, 0)
    assert lib.cn_packed_bytes(h3f, 1) == lib.cn_packed_bytes(h16, 1)
    M = 4133
    assert lib.cn_act_bytes(h3f, M) == lib.cn_act_bytes(h16, M) < lib.cn_act_bytes(h3, M)
    import ctypes
    for kind, idx in ((L_PLANE_Y, 1), (L_PLANE_DA, 2), (L_PLANE_PE, 0), (L_PLANE_MASKS, 0)):
        w3f, w3 = ctypes.c_int(), ctypes.c_int()
        o3f = lib.cn_act_plane(h3f, M, kind, idx, ctypes.byref(w3f))
        o3 = lib.cn_act_plane(h3, M, kind, idx, ctypes.byref(w3))
        assert o3f == o3 >= 0 and w3f.value == w3.value
    assert lib.cn_act_plane(h3f, M, L_PLANE_PELO, 0, None) == -1
    assert lib.cn_act_plane(h3, M, L_PLANE_PELO, 0, None) > 0
    for h in (h16, h3, h3f):
        lib.cn_plan_destroy(h)
    bad = ctypes.c_void_p()
    assert lib.cn_plan_create(3, 1, 256, 10, 4, 256, 4, ctypes.byref(bad)) == -1


L_PLANE_Y, L_PLANE_DA, L_PLANE_PE, L_PLANE_MASKS, L_PLANE_PELO = 0, 1, 2, 4, 6     # include/codenerf.h


@pytest.mark.parametrize("fn", ["cn_mlp_fwd", "cn_mlp_bwd", "cn_mlp_dw"])
def test_sample_guard_rejects_oversized_calls(fn):
    """A call over CN_MAX_SAMPLES samples fails with -1 and a message before
    anything is launched (the kernels index samples with 32-bit integers),
    instead of wrapping silently."""
    import ctypes
    import codenerf_amd._lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("library not built")
    lib = L.load_library()
    h = _plan(lib)
    big = lib.cn_max_samples() + 256
    d = ctypes.c_void_p(16)          # never dereferenced: validation comes first
    if fn == "cn_mlp_fwd":
        rc = lib.cn_mlp_fwd(h, d, d, big, None, None, d, d, d, 0, 64, d, d, d, big, 0, None)
    elif fn == "cn_mlp_bwd":
        rc = lib.cn_mlp_bwd(h, d, d, big, d, d, d, None)
    else:
        rc = lib.cn_mlp_dw(h, d, big, d, d, d, d, d, None)
    assert rc == -1
    assert b"CN_MAX_SAMPLES" in lib.cn_last_error()
    # a workspace laid out for more rows than the guard allows is refused too
    rc = lib.cn_mlp_bwd_rows(h, d, d, 256, d, d, d, big, 0, None)
    assert rc == -1 and b"CN_MAX_SAMPLES" in lib.cn_last_error()
    lib.cn_plan_destroy(h)


def test_hot_kernels_do_not_spill():
    """Every chain / dW kernel of the shipped library keeps its operands in
    registers: a scratch-spilling build (e.g. a compiler change that leaves a
    loop body un-inlined) runs several times slower, so it must not ship
    (tools/kernel_resources.py reads the code object's metadata)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import kernel_resources as kr
    if not os.path.exists(kr.LIB):
        pytest.skip("library not built")
    ks = kr.kernels()
    hot = kr.hot(ks)
    assert len(hot) >= kr.MIN_HOT, len(hot)
    assert not [k for k in hot if k[3] > 0 or k[5]], [k for k in hot if k[3] > 0 or k[5]]
