#!/bin/bash
# round 6 (c): the benchmarked 64 + 64 workload's PSNR tests (64^2 replay and
# 40-epoch horizon; 128^2 x 32 epochs x 2 seeds) and the one-object regime.
export TMPDIR=/tmp
OUT=gpurun_out/r06c
mkdir -p $OUT
timeout -k 10 1150 python -u -m pytest -v -rA --timeout 1100 --timeout-method thread tests/test_gpu_regime_fine.py \
  tests/test_gpu_converge.py > $OUT/pytest_fine_converge.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ge 124 ] && exit $rc
echo r06c done
