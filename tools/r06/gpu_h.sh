#!/bin/bash
# round 6 (h): the weight stream's pieces spread over their issue window
# (tools/r06/patch_spread.py, variants/spread) -- parity of the variant, then
# kbench A/B interleaved against this tree.
export TMPDIR=/tmp
OUT=gpurun_out/r06h
mkdir -p $OUT
CODENERF_MEASURE=1 CODENERF_LIB=variants/spread/libcodenerf_hip.so timeout -k 10 600 python -u -m pytest -x -q \
  --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_planes.py tests/test_gpu_bf16x3f.py \
  tests/test_gpu_bf16x3.py tests/test_gpu_dw.py > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in new spread; do
    case $lib in new) L=;; spread) L=variants/spread/libcodenerf_hip.so;; esac
    for prec in bf16x3f bf16 bf16x3; do
      echo "== rep $rep lib $lib prec $prec" >> $OUT/kb.log
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only fwd,bwd --reps 20 \
        --precision $prec >> $OUT/kb.log 2>&1 || exit 1
    done
  done
done
echo r06h done
