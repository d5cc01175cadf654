"""GPU: the two ABI-3 launch hooks (include/codenerf.h).

* cn_time_next_launch: the next hot launch records the caller's two events
  from its own dispatch (bench.py's per-kernel timers); only that launch.
* cn_stream_wait: a fence-less stream dependency (render.ImageStep's dX / dW
  fork and join): work queued on the waiter after the call sees everything
  the signaller queued before it.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    h = ctypes.CDLL("libamdhip64.so.7")
    h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
    h.hipEventQuery.argtypes = [ctypes.c_void_p]
    h.hipEventDestroy.argtypes = [ctypes.c_void_p]
    return h


def _event(h):
    e = ctypes.c_void_p()
    assert h.hipEventCreateWithFlags(ctypes.byref(e), 0x20000000) == 0     # hipEventDisableSystemFence
    return e


def _fwd_setup(M):
    from golden_util import load, case_params
    from codenerf_amd.model import CodeNeRF
    g = load("c1_32x32_n32")
    dev = torch.device("cuda", 0)
    m = CodeNeRF(3, 1, precision="bf16")
    m.load_state_dict({k: torch.tensor(v) for k, v in case_params(g).items()})
    m = m.to(dev)
    eng = m.engine()
    params = m.param_list()
    eng.ensure_packed(params, bwd=False)
    s = torch.tensor(g["shape_table"][0], device=dev)
    t = torch.tensor(g["texture_table"][0], device=dev)
    blob, _ = eng.latent_fwd(params, s, t)
    gen = torch.Generator().manual_seed(5)
    xyz = (torch.rand(M, 3, generator=gen) * 2 - 1).to(dev)
    vd = torch.nn.functional.normalize(torch.randn(M, 3, generator=gen), dim=-1).to(dev)
    return eng, blob, xyz, vd


def test_time_next_launch_times_one_launch():
    from codenerf_amd import _lib
    L = _lib.lib()
    h = _hip()
    eng, blob, xyz, vd = _fwd_setup(1 << 18)
    assert L.cn_time_next_launch(_event(h), None) != 0          # both events or none
    s, e = _event(h), _event(h)
    assert L.cn_time_next_launch(s, e) == 0
    eng.mlp_fwd(blob, xyz.shape[0], xyz=xyz, viewdir=vd)        # timed: the chain launch
    eng.mlp_fwd(blob, xyz.shape[0], xyz=xyz, viewdir=vd)        # untimed: the hook was consumed
    s2, e2 = _event(h), _event(h)
    assert L.cn_time_next_launch(s2, e2) == 0
    eng.mlp_fwd(blob, xyz.shape[0], xyz=xyz, viewdir=vd)        # timed again
    torch.cuda.synchronize()
    for a, b in ((s, e), (s2, e2)):
        ms = ctypes.c_float()
        assert h.hipEventElapsedTime(ctypes.byref(ms), a, b) == 0
        assert 0.0 < ms.value < 1000.0
    assert L.cn_time_next_launch(None, None) == 0               # clears


def test_stream_wait_orders_two_streams():
    from codenerf_amd import _lib
    L = _lib.lib()
    eng, blob, xyz, vd = _fwd_setup(1 << 20)
    dev = xyz.device
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    ref_sig, _ = eng.mlp_fwd(blob, xyz.shape[0], xyz=xyz, viewdir=vd)
    torch.cuda.synchronize()
    for _ in range(3):
        sig = torch.full_like(ref_sig, float("nan"))
        sig2 = torch.empty_like(ref_sig)
        torch.cuda.synchronize()
        # main: a ~1 ms chain launch writes sig; side copies sig after the wait
        eng.mlp_fwd(blob, xyz.shape[0], xyz=xyz, viewdir=vd, sigma=sig)
        assert L.cn_stream_wait(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(main.cuda_stream)) == 0
        with torch.cuda.stream(side):
            sig2.copy_(sig)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(sig2.cpu().numpy(), ref_sig.cpu().numpy())
