"""Import name of the package whose sources live in ``code-nerf_amd/`` (the
directory name the build layout prescribes is not a Python identifier).

The package search path is pointed at that directory, so ``codenerf_amd.model``,
``codenerf_amd.render`` ... are the modules in ``code-nerf_amd/`` loaded by the
normal import machinery (no exec, no copies); this file only re-exports what
``code-nerf_amd/__init__.py`` exports.
"""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "code-nerf_amd")]

from ._lib import CnError, HipUnavailable, LIB_PATH  # noqa: E402,F401

__all__ = ["HipUnavailable", "CnError", "LIB_PATH"]
