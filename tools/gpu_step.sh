#!/bin/bash
# One GPU call of the build loop: kernel timings (tools/kbench.py) per
# precision and library variant, optional bench lines, targeted tests (fail
# fast), then optionally the full check (tools/gpu_check.sh).
#   bash tools/gpu_step.sh TAG "pytest targets" [full]
# env: KB_PRECS (default "bf16 bf16x3"), KB_VARIANTS (library variants
#      code-nerf_amd/libcodenerf_hip_<v>.so besides the default, e.g. "d4"),
#      BENCH_ARGS (";"-separated bench.py argument sets, one line each)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=$1; TARGETS=$2; FULL=$3
for p in ${KB_PRECS-bf16 bf16x3}; do
  for v in default $KB_VARIANTS; do
    lib=""; [ "$v" != default ] && lib=$R/code-nerf_amd/libcodenerf_hip_$v.so
    CODENERF_MEASURE=1 CODENERF_LIB=$lib timeout -k 10 180 python -u tools/kbench.py --precision $p --only fwd,bwd,dw > $O/kb_${TAG}_${p}_$v.log 2>&1 \
      || { echo "kbench $p $v failed"; tail -20 $O/kb_${TAG}_${p}_$v.log; exit 1; }
    echo "$v $(tail -1 $O/kb_${TAG}_${p}_$v.log)"
  done
done
IFS=';' read -ra BA <<< "$BENCH_ARGS"
i=0
for a in "${BA[@]}"; do
  [ -z "$a" ] && continue
  timeout -k 10 400 python -u bench.py $a > $O/bench_${TAG}_$i.log 2>&1 || { echo "bench $a failed"; tail -20 $O/bench_${TAG}_$i.log; exit 1; }
  echo "bench $a: $(tail -1 $O/bench_${TAG}_$i.log | cut -c1-400)"
  i=$((i+1))
done
if [ -n "$TARGETS" ]; then
  timeout -k 10 1000 python -u -m pytest $TARGETS -x -v -s --timeout 900 --timeout-method thread > $O/pt_$TAG.log 2>&1 \
    || { echo "targeted tests failed"; grep -E "PASS|FAIL|Error|error|assert" $O/pt_$TAG.log | tail -40; exit 1; }
  grep -E "passed|failed" $O/pt_$TAG.log | tail -2
fi
if [ -n "$FULL" ]; then bash tools/gpu_check.sh $TAG || exit 1; fi
