#!/bin/bash
# round 4 (l): one-object test with the reference-on-GPU floor; bf16x3 chain stall counters
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread \
  tests/test_gpu_converge.py::test_early_train_psnr_matches_reference_at_each_precision > $O/pytest_converge.log 2>&1
echo "pytest rc=$?"
grep "horizon\|replayable" $O/pytest_converge.log | cut -c1-400
bash tools/gpu_stalls.sh r04l/x3 bf16x3 || exit 1
bash tools/gpu_stalls.sh r04l/b16 bf16 || exit 1
echo r04l done
