#!/bin/bash
# GPU-box profiling recipe (run through gpurun from the repo root):
#   tools/gpu_profile.sh <tag> [bench args...]
# Writes under gpurun_out/<tag>/:
#   stats/      rocprofv3 --kernel-trace --stats
#   mfma/       SQ/GRBM counters (MFMA busy cycles, wave cycles, clocks)
#   fetch/      FETCH_SIZE      (its own pass: TCC slots)
#   write/      WRITE_SIZE      (its own pass)
# Every GPU step has its own time limit; a timeout or a signal ends the script.
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
BENCH="bench.py --no-cpu-baseline --no-fp32 --steps 20 --warmup 5 $*"

run() {
  "$@"
  rc=$?
  if [ $rc -ge 124 ]; then
    echo "FATAL rc=$rc: $*" >&2
    exit $rc
  fi
  return 0
}

run timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- python3 $BENCH > "$OUT/stats.log" 2>&1
run timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/mfma" -o run --output-format csv -- python3 $BENCH > "$OUT/mfma.log" 2>&1
run timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $BENCH > "$OUT/fetch.log" 2>&1
run timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $BENCH > "$OUT/write.log" 2>&1
echo "profile $TAG done"
