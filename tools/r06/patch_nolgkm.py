# Timing ablation (results invalid): the bf16x3 forward's counted A-fragment
# waits dropped (each MFMA may read the fragment register before its LDS read
# returns -- the previous contents: realistic operand values, so the clock
# stays that of real data).  Measures what waiting on the fragment reads costs.
import sys
p = sys.argv[1] + "/chain.hip"
s = open(p).read()
old = '''          asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Abuf[g % (kPF + 1)]) : "n"(younger));'''
new = '''          if constexpr (BWD) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(Abuf[g % (kPF + 1)]) : "n"(younger));
          else asm volatile("" : "+v"(Abuf[g % (kPF + 1)]));'''
assert s.count(old) == 1
s = s.replace(old, new)
open(p, "w").write(s)
print("nolgkm")
