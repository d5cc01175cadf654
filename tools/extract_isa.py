"""Disassemble the gfx950 code object embedded in a hipcc object file or
shared library (clang offload bundle in .hip_fatbin):
  python tools/extract_isa.py <file.o|.so> <out.s>"""
import struct
import subprocess
import sys

data = open(sys.argv[1], "rb").read()
magic = b"__CLANG_OFFLOAD_BUNDLE__"
pos = data.find(magic)
out = []
while pos >= 0:
    n = struct.unpack_from("<Q", data, pos + 24)[0]
    p = pos + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", data, p)
        triple = data[p + 24:p + 24 + tl].decode()
        p += 24 + tl
        if "gfx950" in triple:
            out.append(data[pos + off:pos + off + size])
    pos = data.find(magic, pos + 32)
for i, blob in enumerate(out):
    fn = f"/tmp/_co{i}.elf"
    open(fn, "wb").write(blob)
    s = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", fn],
                       capture_output=True, text=True).stdout
    open(sys.argv[2] if i == 0 else f"{sys.argv[2]}.{i}", "w").write(s)
    print(f"code object {i}: {len(blob)} B -> {len(s.splitlines())} lines")
