#!/bin/bash
# round 4 (o): fence-less stream fork/join and timers, latent_fwd float4 rows,
# fine-loss z in LDS -- full gpu suite, smoke, bench, step timeline
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAILED\|Error" $O/pytest_gpu.log | head; }
grep -n "passed\|failed" $O/pytest_gpu.log | tail -2
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
bash tools/gpu_profile.sh r04o/prof || exit 1
echo r04o done
