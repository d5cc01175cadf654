#!/bin/bash
# round 4 (y): emulation of seeds 3 and 6 (where bf16x3 left the reference early): which operand split holds them?
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04y; mkdir -p $O
for s in 3 6; do
  EMU_DEVICE=cuda EMU_THREADS=16 EMU_ONLY=f_path,bf16,x3_kernel,x3_kernel_dwall,s3_dwall timeout -k 10 400 python -u tools/split_emu.py many 320 $s > $O/emu_seed$s.log 2>&1 || exit 1
  grep "epoch-mean" $O/emu_seed$s.log | cut -c1-30
done
echo r04y done
