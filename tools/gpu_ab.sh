#!/bin/bash
# Interleaved A/B of two bench.py argument sets on one box:
#   tools/gpu_ab.sh <tag> <reps> "<args A>" "<args B>"
# Appends one JSON line per run to gpurun_out/<tag>_A.jsonl / _B.jsonl.
TAG=$1
REPS=$2
A=$3
B=$4
mkdir -p gpurun_out
for i in $(seq 1 "$REPS"); do
  timeout -k 10 180 python3 bench.py --no-cpu-baseline $A >> "gpurun_out/${TAG}_A.jsonl" || exit $?
  timeout -k 10 180 python3 bench.py --no-cpu-baseline $B >> "gpurun_out/${TAG}_B.jsonl" || exit $?
done
echo "ab $TAG done"
