# bf16x3 chains: A-fragment read-ahead distance kPF (variant name pf<N>); the
# weight-stream pieces' spread shrinks so a chunk's G pieces still fit the
# first window (kChunkBlocks - kPF blocks).  Timing A/B; results unchanged.
import os
import re
import sys
d = sys.argv[1]
name = os.path.basename(os.path.dirname(os.path.abspath(d)))
n = int(re.match(r"pf(\d+)", name).group(1))
p = d + "/chain.hip"
s = open(p).read()


def sub(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


sub("static constexpr int kPF = kX3 ? 3 : 2;", f"static constexpr int kPF = kX3 ? {n} : 2;")
sub("static constexpr int kSpread = kX3 ? kChunkBlocks / G : 0;",
    "static constexpr int kSpread = kX3 ? (kChunkBlocks / G < (kChunkBlocks - kPF - 1) / (G - 1) ? kChunkBlocks / G "
    ": (kChunkBlocks - kPF - 1) / (G - 1)) : 0;")
open(p, "w").write(s)
print("kPF", n)
