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
    assert lib.cn_abi_version() == 1


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
