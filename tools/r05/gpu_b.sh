#!/bin/bash
# round 5 (b): the trace against the kernel-faithful emulation (latent-path
# bias sums from the bf16 dA plane), and seed-3 emulation trajectories of it
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r04x3.so CODENERF_MEASURE=1
timeout -k 10 400 python -u tools/x3_trace.py $O/trace_seed3_db.json 3 0 104 > $O/trace_seed3_db.log 2>&1 || { tail -30 $O/trace_seed3_db.log; exit 1; }
grep -A32 "step 104" $O/trace_seed3_db.log | head -34
EMU_DEVICE=cuda EMU_THREADS=16 EMU_ONLY=x3_kernel,x3_kdb,x3_ksdb timeout -k 10 600 python -u tools/split_emu.py many 320 3 > $O/emu_seed3.log 2>&1 || { tail -30 $O/emu_seed3.log; exit 1; }
grep "epoch-mean" $O/emu_seed3.log | cut -c1-400
echo r05b done
