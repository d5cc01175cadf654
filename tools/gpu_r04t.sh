#!/bin/bash
# round 4 (t): final tree -- full gpu suite, smoke, default bench, C3 / C4 / C4eval
# lines, profile (kernel stats + MFMA + FETCH + WRITE passes) of the C2 step
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAILED\|Error" $O/pytest_gpu.log | head; }
grep -n "passed\|failed" $O/pytest_gpu.log | tail -1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
for c in c3 c4 c4eval; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline --no-fp32 --steps 10 --warmup 3 > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log | cut -c1-160
done
bash tools/gpu_profile.sh r04t/prof || exit 1
echo r04t done
