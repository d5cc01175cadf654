#!/bin/bash
# round 5 (d): per-tensor trace of HIP bf16x3 (16x16x32 chains) vs the
# kernel-faithful emulation (OPS_BF16X3_DB) around seed 3's exit, then the
# seed-3 long-horizon record of the built library
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 420 python -u tools/x3_trace.py $O/trace_seed3.json 3 96 104 > $O/trace_seed3.log 2>&1 || { tail -30 $O/trace_seed3.log; exit 1; }
grep -B2 -A32 "step 104" $O/trace_seed3.log | head -40
timeout -k 10 600 python -u tools/regime_seeds.py $O/seed3.json 3 > $O/seed3.log 2>&1 || { tail -30 $O/seed3.log; exit 1; }
grep -E "first epoch|horizon" $O/seed3.log | cut -c1-400
echo r05d done
