#!/bin/bash
# One GPU call of the build loop: targeted tests (fail fast), kernel timings
# (tools/kbench.py) per precision, then the full check (tools/gpu_check.sh).
#   bash tools/gpu_step.sh TAG "pytest targets" [full]
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=$1; TARGETS=$2; FULL=$3
if [ -n "$TARGETS" ]; then
  timeout -k 10 900 python -u -m pytest $TARGETS -x -v -s --timeout 900 --timeout-method thread > $O/pt_$TAG.log 2>&1 \
    || { echo "targeted tests failed"; grep -E "PASS|FAIL|Error|error|assert" $O/pt_$TAG.log | tail -40; exit 1; }
  grep -E "passed|failed" $O/pt_$TAG.log | tail -2
fi
for p in bf16 bf16x3; do
  timeout -k 10 180 python -u tools/kbench.py --precision $p --only fwd,bwd,dw > $O/kb_${TAG}_$p.log 2>&1 || { echo "kbench $p failed"; tail -20 $O/kb_${TAG}_$p.log; exit 1; }
  tail -1 $O/kb_${TAG}_$p.log
done
if [ -n "$FULL" ]; then bash tools/gpu_check.sh $TAG || exit 1; fi
