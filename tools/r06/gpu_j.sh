#!/bin/bash
# round 6 (j): the train-PSNR test files on the current kernels (the layout,
# early-issue and spread changes alter every rounding order, so the chaotic
# trajectories are re-run, not assumed).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06j}
mkdir -p $OUT
timeout -k 10 1150 python -u -m pytest -v -rA --timeout 1100 --timeout-method thread tests/test_gpu_regime.py \
  tests/test_gpu_regime_fine.py tests/test_gpu_converge.py > $OUT/pytest_psnr.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ge 124 ] && exit $rc
echo r06j done
