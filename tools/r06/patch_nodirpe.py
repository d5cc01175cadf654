# Timing probe (results invalid): the forward prologue's view-direction
# encoding without its 7 sincosf per lane (sin / cos replaced by the scaled
# direction component itself) -- what a per-ray precompute could save.
import sys
p = sys.argv[1] + "/chain.hip"
s = open(p).read()
old = '''        const float v = (comp == 0 ? d[0] : comp == 1 ? d[1] : d[2]) * (float)(1 << oct);
        if constexpr (kBf16 && !kX3) sincos_turns(v, sn, cs);
        else sincosf(v, &sn, &cs);'''
new = '''        const float v = (comp == 0 ? d[0] : comp == 1 ? d[1] : d[2]) * (float)(1 << oct);
        sn = v * 0.5f; cs = v * 0.25f;'''
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
print("nodirpe")
