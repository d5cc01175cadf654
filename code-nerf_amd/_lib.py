"""ctypes binding of the C ABI in include/codenerf.h (libcodenerf_hip.so).

This is the product path's only way to compute: if the library or a HIP device
is missing, every entry point raises ``HipUnavailable`` -- there is no CPU
fallback.  torch is imported first so the process already holds torch's HIP
runtime (SONAME libamdhip64.so.7) when the library is loaded.
"""
import ctypes
import os

import torch

LIB_NAME = "libcodenerf_hip.so"
_IN_TREE = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# CODENERF_LIB selects another build of the same ABI -- a measurement-only
# kernel variant built from a patched copy of csrc/ (tools/kbench.py A/Bs).
# Such a build is loaded only when CODENERF_MEASURE=1 is set as well: the
# product path (tests, smoke, bench) always runs the in-tree library.
LIB_PATH = os.environ.get("CODENERF_LIB") or _IN_TREE

ABI_VERSION = 3
CN_FP32 = 0
CN_BF16 = 1
CN_BF16X3 = 2
CN_BF16X3F = 3      # bf16x3 forward chains, bf16 backward (include/codenerf.h)


class HipUnavailable(RuntimeError):
    pass


class CnError(RuntimeError):
    pass


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_D = ctypes.c_double
_Z = ctypes.c_size_t

_SIGS = {
    "cn_abi_version": (_I, []),
    "cn_last_error": (ctypes.c_char_p, []),
    "cn_time_next_launch": (_I, [_P, _P]),
    "cn_stream_wait": (_I, [_P, _P]),
    "cn_plan_create": (_I, [_I, _I, _I, _I, _I, _I, _I, ctypes.POINTER(_P)]),
    "cn_plan_destroy": (None, [_P]),
    "cn_plan_num_params": (_I, [_P]),
    "cn_plan_num_inject": (_I, [_P]),
    "cn_pad_samples": (_I, [_P, _I]),
    "cn_max_samples": (_I, []),
    "cn_act_bytes_per_sample": (_Z, [_P]),
    "cn_packed_bytes": (_Z, [_P, _I]),
    "cn_blob_floats": (_Z, [_P]),
    "cn_act_bytes": (_Z, [_P, _I]),
    "cn_dw_ws_bytes": (_Z, [_P, _I]),
    "cn_act_plane": (ctypes.c_longlong, [_P, _I, _I, _I, ctypes.POINTER(_I)]),
    "cn_pack_weights": (_I, [_P, _P, _P, _P, _P]),
    "cn_latent_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P]),
    "cn_mlp_fwd": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _I, _P]),
    "cn_mlp_bwd": (_I, [_P, _P, _P, _I, _P, _P, _P, _P]),
    "cn_mlp_fwd_codes": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _I, _I, _P]),
    "cn_mlp_bwd_codes": (_I, [_P, _P, _P, _I, _P, _P, _P, _I, _I, _P]),
    "cn_mlp_dw": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P]),
    "cn_mlp_bwd_rows": (_I, [_P, _P, _P, _I, _P, _P, _P, _I, _I, _P]),
    "cn_mlp_dw_rows": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _I, _I, _P, _P]),
    "cn_mlp_dbias": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    "cn_latent_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P]),
    "cn_get_rays": (_I, [_I, _I, _D, _I, _P, _P, _P, _P]),
    "cn_sample_points": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "cn_composite_fwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "cn_composite_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "cn_render_loss": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P]),
    "cn_sample_pdf": (_I, [_P, _P, _I, _I, _I, _P, _I, _P, _P]),
    "cn_render_loss_fine": (_I, [_P, _P, _P, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P,
                                 _P]),
    "cn_adamw_step": (_I, [_I, _P, _P, _P, _P, _P, _P, _D, _D, _D, _D, _I, _P]),
    "cn_adamw_step_zero_grad": (_I, [_I, _P, _P, _P, _P, _P, _P, _D, _D, _D, _D, _I, _P]),
    "cn_clock_probe": (_I, [_P, _I, _I, ctypes.c_uint, _P]),
}

EXPORTED = tuple(_SIGS)
_lib = None


def load_library(path=LIB_PATH):
    """Load and type the shared library (no device needed)."""
    if not os.path.exists(path):
        raise HipUnavailable(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    variant = os.path.abspath(path) != os.path.abspath(_IN_TREE)
    if variant and os.environ.get("CODENERF_MEASURE") != "1":
        raise HipUnavailable(f"{path} is not the in-tree library: a measurement variant loads only with "
                             "CODENERF_MEASURE=1")
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if variant:          # an older A/B build may lack a newer query
                continue
            raise HipUnavailable(f"{path} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    if lib.cn_abi_version() != ABI_VERSION:
        raise HipUnavailable("libcodenerf_hip.so ABI version mismatch")
    return lib


def lib():
    """The loaded library; requires a visible HIP device."""
    global _lib
    if _lib is None:
        if not torch.cuda.is_available():
            raise HipUnavailable("no HIP device visible: the CodeNeRF MI355X path has no CPU fallback")
        _lib = load_library()
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().cn_last_error().decode(errors="replace")
        raise CnError(f"{what}: {msg}" if what else msg)


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
