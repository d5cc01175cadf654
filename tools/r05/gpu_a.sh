#!/bin/bash
# round 5 (a): per-tensor trace of HIP bf16x3 vs its emulation on regime seed 3; a bench line
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 500 python -u tools/x3_trace.py $O/trace_seed3.json 3 0 104 120 > $O/trace_seed3.log 2>&1 || { tail -30 $O/trace_seed3.log; exit 1; }
grep -A30 "step 104" $O/trace_seed3.log | head -40
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
echo r05a done
