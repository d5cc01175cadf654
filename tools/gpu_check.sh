#!/bin/bash
# One GPU call: gpu tests, smoke, bench, rocprof kernel stats.  Each GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $OUT
TAG=${1:-run}
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke_$TAG.log; exit 1; }
tail -2 $OUT/smoke_$TAG.log
timeout -k 10 300 python -u bench.py > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log
