# timing probe (results invalid for parity): the bf16x3 forward's positional
# encoding on the transcendental unit (sincos_turns) instead of sincosf
import sys
p = sys.argv[1] + "/chain.hip"
s = open(p).read()
old = "if constexpr (kBf16 && !kX3) sincos_turns(v, sn, cs);"
assert s.count(old) == 2
s = s.replace(old, "if constexpr (kBf16) sincos_turns(v, sn, cs);")
open(p, "w").write(s)
