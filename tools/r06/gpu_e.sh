#!/bin/bash
# round 6 (e): forward chains with the weight stream issued before the
# prologue -- parity of the new tree (fp32 / bf16 / bf16x3 / bf16x3f forward
# paths, planes), then kbench A/B interleaved: round-start library
# (variants/base.so), this tree, and a timing-only probe with the bf16x3 PE
# on the transcendental unit (variants/hwsc).
export TMPDIR=/tmp
OUT=gpurun_out/r06e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_planes.py tests/test_gpu_bf16x3f.py tests/test_gpu_bf16x3.py > $OUT/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in base new hwsc; do
    case $lib in base) L=variants/base.so;; new) L=;; hwsc) L=variants/hwsc/libcodenerf_hip.so;; esac
    for prec in bf16x3f bf16; do
      [ $lib = hwsc ] && [ $prec = bf16 ] && continue
      echo "== rep $rep lib $lib prec $prec" >> $OUT/kb.log
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only fwd,bwd --reps 20 \
        --precision $prec >> $OUT/kb.log 2>&1 || exit 1
    done
  done
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
echo r06e done
