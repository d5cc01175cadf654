"""Register / scratch / LDS use of every kernel in the gfx950 code object of
libcodenerf_hip.so (or a hipcc .o), read from the code object's metadata
notes (llvm-readelf --notes).  Used by __graft_entry__.build() and the CPU
tests as a guard: a shipped chain or dW kernel that spills to scratch runs
several times slower (a compiler change that un-inlines a loop body puts the
register arrays in scratch), so the build refuses it.

  python tools/kernel_resources.py [path]        -> table; exit 1 on spills
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "code-nerf_amd", "libcodenerf_hip.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(path):
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = data.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple:
                yield data[pos + off:pos + off + size]
        pos = data.find(magic, pos + 32)


def kernels(path=LIB):
    """[(name, vgpr, agpr, scratch bytes per lane, lds bytes, uses dynamic stack)]"""
    out = []
    for blob in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".elf") as f:
            f.write(blob)
            f.flush()
            notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
        # one kernel = one entry of the amdhsa.kernels list ("  - .agpr_count:")
        for blk in re.split(r"\n  - (?=\.agpr_count:)", notes)[1:]:
            m = re.search(r"^\s*\.name:\s+(\S+)", blk, re.M)
            if not m:
                continue
            name = m.group(1)
            g = lambda k: int((re.search(rf"^\s*\.{k}:\s+(\d+)", blk, re.M) or [0, -1])[1])
            if g("vgpr_count") < 0:
                continue
            dyn = re.search(r"^\s*\.uses_dynamic_stack:\s+(\w+)", blk, re.M)
            out.append((name, g("vgpr_count"), g("agpr_count"), g("private_segment_fixed_size"),
                        g("group_segment_fixed_size"), bool(dyn and dyn.group(1) in ("true", "1"))))
    return out


def spills(path=LIB):
    """kernels with fixed scratch or a dynamic stack"""
    return [k for k in kernels(path) if k[3] > 0 or k[5]]


def hot(ks):
    """the hot kernels of a kernel list: chain (forward / dX) and dW"""
    return [k for k in ks if re.search(r"chain_kernel|dw_kernel", k[0])]


# hot kernels the library must contain: 6 chain sets (fp32 / bf16 / bf16x3 x
# (3,1) / (2,1)) x 5 chain kernels (fwd train / infer / codes, dX train /
# codes) + the 2 dW instantiations (bf16 planes, fp32 planes)
MIN_HOT = 6 * 5 + 2


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else LIB
    ks = kernels(path)
    for name, v, a, s, l, dyn in ks:
        print(f"{v:4d} vgpr {a:4d} agpr {s:6d} B scratch {l:7d} B lds {'dyn-stack ' if dyn else ''} {name}")
    bad = [k for k in ks if k[3] > 0 or k[5]]
    print(f"{len(ks)} kernels, {len(bad)} with scratch")
    sys.exit(1 if bad else 0)
