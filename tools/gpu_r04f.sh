#!/bin/bash
# round 4 (f): paired dW staging -- parity of dW, kbench A/B, then the PSNR tests
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04f; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dw.py > $O/pytest_dw.log 2>&1
for rep in 1 2; do
  for v in in-tree dw_nopair; do
    if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
    for p in bf16 bf16x3; do
      CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 240 python -u tools/kbench.py --precision $p --only dw --reps 20 > $O/kbdw_${p}_${v}_$rep.json 2> $O/kbdw_${p}_${v}_$rep.log
    done
  done
done
timeout -k 10 1000 python -u -m pytest -v -s --timeout 900 --timeout-method thread \
  tests/test_gpu_converge.py::test_early_train_psnr_matches_reference_at_each_precision tests/test_gpu_regime.py \
  tests/test_gpu_regime_fine.py > $O/pytest_psnr.log 2>&1
echo "psnr rc=$?"
