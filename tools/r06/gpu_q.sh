#!/bin/bash
# round 6 (q): does operand data move the bf16x3 forward's time (matrix-core
# power -> clock)?  kbench fwd with the weights as trained vs all zero, on the
# in-tree library and on the no-LDS-DMA ablation; 3 interleaved reps.
export TMPDIR=/tmp
OUT=gpurun_out/r06q
mkdir -p $OUT
for rep in 1 2 3; do
  for v in base abl_nodma; do
    for s in 1 0; do
      case $v in base) L=;; *) L=variants/$v/libcodenerf_hip.so;; esac
      echo "== rep $rep lib $v scale $s" >> $OUT/kb.log
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only fwd --reps 20 \
        --precision bf16x3f --weight-scale $s >> $OUT/kb.log 2>&1 || exit 1
    done
  done
done
echo done
