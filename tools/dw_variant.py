"""Measurement-only dW variants (capi.hip + dw.hip from a patched copy of
csrc/, linked with the in-tree chain objects): libcodenerf_hip_<name>.so,
loaded by tools/kbench.py only with CODENERF_MEASURE=1 CODENERF_LIB=...

  python tools/dw_variant.py NAME 'old text' 'new text' ['old' 'new' ...]
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "code-nerf_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-Wall", "-Wno-unused-variable",
         "-Wno-unused-function"]


def main():
    name, subs = sys.argv[1], sys.argv[2:]
    tmp = tempfile.mkdtemp()
    src = os.path.join(tmp, "pkg", "csrc")      # capi.hip includes ../../include/codenerf.h
    shutil.copytree(CSRC, src, ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
    p = os.path.join(src, "dw.hip")
    s = open(p).read()
    for old, new in zip(subs[0::2], subs[1::2]):
        if old not in s:
            sys.exit(f"pattern not found: {old!r}")
        s = s.replace(old, new)
    open(p, "w").write(s)
    obj = os.path.join(tmp, "capi.o")
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-c", os.path.join(src, "capi.hip"), "-o", obj], check=True)
    insts = sorted(os.path.join(CSRC, "build", f) for f in os.listdir(os.path.join(CSRC, "build"))
                   if f.startswith("inst_") and f.endswith(".o"))
    out = os.path.join(REPO, "code-nerf_amd", f"libcodenerf_hip_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, obj, *insts],
                   check=True)
    print("built", out)


if __name__ == "__main__":
    main()
