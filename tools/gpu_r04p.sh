#!/bin/bash
# round 4 (p): kbench of the chain kernels on this build (is the step's slower chain the kernel or the box?)
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
for p in bf16 bf16x3; do
  timeout -k 10 240 python -u tools/kbench.py --precision $p --only fwd,bwd --reps 10 > $O/kb_$p.json 2> $O/kb_$p.log || exit 1
  cat $O/kb_$p.json
done
rocm-smi --showclocks --showpower > $O/smi.txt 2>&1; head -40 $O/smi.txt
