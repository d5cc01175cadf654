#!/bin/bash
# round 6 (l): the bf16x3 forward tile pipeline (variants/pipe: TRAIN_HI kernel only)
# against the in-tree library, kbench fwd of the bf16x3f plan, 3 interleaved reps.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06l}
mkdir -p $OUT
for rep in 1 2 3; do
  for v in base ${VARIANTS:-pipe}; do
    case $v in base) L=;; *) L=variants/$v/libcodenerf_hip.so;; esac
    echo "== rep $rep lib $v" >> $OUT/kb.log
    CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only ${ONLY:-fwd} --reps 20 \
      --precision ${PREC:-bf16x3f} >> $OUT/kb.log 2>&1 || exit 1
  done
done
echo done
