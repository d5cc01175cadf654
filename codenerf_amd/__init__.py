"""Import shim: the package sources live in ``code-nerf_amd/`` (a directory
name Python cannot import directly); this redirects the package path there."""
import os as _os

__path__ = [_os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "code-nerf_amd")]
_init = _os.path.join(__path__[0], "__init__.py")
with open(_init) as _f:
    exec(compile(_f.read(), _init, "exec"))
