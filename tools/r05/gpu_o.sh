#!/bin/bash
# round 5 (o): profiles of the final tree -- C2 bf16 step (kernel stats, MFMA,
# FETCH, WRITE passes) and the bf16x3 step (kernel stats), stall counters
export TMPDIR=/tmp
bash tools/gpu_profile.sh r05o/prof || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05o/x3stats -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-fp32 --steps 20 --warmup 5 --precision bf16x3 > gpurun_out/r05o/x3stats.log 2>&1 || exit 1
bash tools/gpu_stalls.sh r05o/b16 bf16 || exit 1
bash tools/gpu_stalls.sh r05o/x3 bf16x3 || exit 1
python3 tools/prof_summary.py gpurun_out/r05o/prof r05o c2 > gpurun_out/r05o/kernels.md 2>&1 || true
python3 tools/timeline.py gpurun_out/r05o/prof/stats 2 > gpurun_out/r05o/timeline.md 2>&1 || true
echo r05o done
