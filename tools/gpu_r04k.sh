#!/bin/bash
# round 4 (k): the PSNR regime tests against the reference replayed on the GPU
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -v -s --timeout 1000 --timeout-method thread tests/test_gpu_regime.py tests/test_gpu_regime_fine.py > $O/pytest_regime.log 2>&1
echo "pytest rc=$?"
tail -3 $O/pytest_regime.log
