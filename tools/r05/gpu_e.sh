#!/bin/bash
# round 5 (e): stall / issue counters of the 16x16x32 bf16x3 chains and the bf16 chains
export TMPDIR=/tmp
mkdir -p gpurun_out/r05e
bash tools/gpu_stalls.sh r05e/x3 bf16x3 || exit 1
bash tools/gpu_stalls.sh r05e/b16 bf16 || exit 1
echo r05e done
