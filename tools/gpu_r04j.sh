#!/bin/bash
# round 4 (j): the built bf16x3 emulated exactly (dir-PE dW columns hi only)
# with / without the dW upstream-gradient split, three seeds, 40 epochs of the
# many-object regime (torch fp32 on the GPU); C5 bench line; bf16x3 C2 profile
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04j; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
for s in 0 1 2; do
  EMU_DEVICE=cuda EMU_THREADS=16 EMU_ONLY=f_path,s3_dwx,x3_kernel,s3_dwall,x3_kernel_dwall,chain_s3 run timeout -k 10 300 python -u tools/split_emu.py many 320 $s > $O/emu_seed$s.log 2>&1
  grep "epoch-mean" $O/emu_seed$s.log | cut -c1-40
done
run timeout -k 10 400 python -u bench.py --config c5 --no-cpu-baseline --steps 4 --warmup 2 > $O/bench_c5.log 2>&1
tail -1 $O/bench_c5.log | cut -c1-250
run bash tools/gpu_profile.sh r04j/profx --precision bf16x3
echo r04j done
