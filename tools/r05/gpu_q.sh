#!/bin/bash
# round 5 (q): the final tree, clean rebuild -- full gpu suite, smoke, default bench, C3 / C4 / C4eval / C5 lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -n "passed\|failed" $O/pytest_gpu.log | tail -1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ $rc -eq 0 ] || grep -n "FAILED" $O/pytest_gpu.log | head
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
for c in c3 c4 c4eval c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-fp32 --steps 10 --warmup 3 > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
  tail -1 $O/bench_$c.log | cut -c1-160
done
echo r05q done
