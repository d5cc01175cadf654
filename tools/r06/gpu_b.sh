#!/bin/bash
# round 6 (b): train-PSNR parity in the many-object regime (64^2, 64 samples):
# two epochs vs the CPU replay; 40 epochs x seeds 0-7 vs the reference on the
# GPU (bf16x3 over the fp32 horizon; seed 3 the recorded miss); the converged
# tail criterion (bf16x3, bf16x3f); same-weights render; the seed-3 diagnostic.
export TMPDIR=/tmp
OUT=gpurun_out/r06b
mkdir -p $OUT
timeout -k 10 1150 python -u -m pytest -v -rA --timeout 1100 --timeout-method thread tests/test_gpu_regime.py \
  > $OUT/pytest_regime.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -ge 124 ] && exit $rc
echo r06b done
