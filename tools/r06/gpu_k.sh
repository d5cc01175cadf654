#!/bin/bash
# round 6 (k): timing ablations of the bf16x3 forward chain (tools/r06/patch_ablate.py;
# results invalid, timing only): kbench fwd of the bf16x3f plan, in-tree vs
# no LDS-DMA / no DMA + no barrier / no tile epilogue / all three, two
# interleaved repetitions.
export TMPDIR=/tmp
OUT=gpurun_out/r06k
mkdir -p $OUT
for rep in 1 2; do
  for v in base abl_nodma abl_nobar abl_noepi abl_floor; do
    case $v in base) L=;; *) L=variants/$v/libcodenerf_hip.so;; esac
    echo "== rep $rep lib $v" >> $OUT/kb.log
    CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only fwd --reps 20 \
      --precision bf16x3f >> $OUT/kb.log 2>&1 || exit 1
  done
done
echo r06k done
