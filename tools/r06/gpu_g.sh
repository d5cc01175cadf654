#!/bin/bash
# round 6 (f): explicit 16-B prologue stores (exact kProStores) + early weight-stream issue in the backward chains
# : every plane / dW / codes / config parity test, then
# kbench A/B against the r06f library (variants/r06f.so), then the bench.
export TMPDIR=/tmp
OUT=gpurun_out/r06g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_planes.py \
  tests/test_gpu_dw.py tests/test_gpu_parity.py tests/test_gpu_bf16x3.py tests/test_gpu_bf16x3f.py \
  tests/test_gpu_configs.py tests/test_gpu_train.py tests/test_gpu_fine.py > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in base new; do
    case $lib in base) L=variants/r06f.so;; new) L=;; esac
    for prec in bf16x3f bf16 bf16x3; do
      echo "== rep $rep lib $lib prec $prec" >> $OUT/kb.log
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only fwd,bwd,dw --reps 20 \
        --precision $prec >> $OUT/kb.log 2>&1 || exit 1
    done
  done
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
echo r06g done
