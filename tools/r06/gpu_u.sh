#!/bin/bash
# round 6 (u): final tree -- the GPU suite except the train-PSNR files (those:
# gpu_j.sh, r06m), smoke, bench.
export TMPDIR=/tmp
OUT=gpurun_out/r06u
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_regime.py --deselect tests/test_gpu_regime_fine.py --deselect tests/test_gpu_converge.py \
  > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
echo r06u done
