"""codenerf_amd: the CodeNeRF render/train hot path as hand-written HIP kernels
for MI355X (gfx950), behind the reference's Python API.

Import as ``codenerf_amd`` (the sources live in ``code-nerf_amd/``).
"""
from ._lib import HipUnavailable, CnError, LIB_PATH  # noqa: F401

__all__ = ["HipUnavailable", "CnError", "LIB_PATH"]
