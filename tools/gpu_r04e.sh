#!/bin/bash
# round 4 (e): does the bf16x3 dW X split change the many-object trajectory?
# fp32 (two summation orders), bf16x3 with the split (in-tree) and without it
# (the round-start build), seeds 0-2, 40 epochs each, one process per run.
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04e; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
for s in 0 1 2; do
  run timeout -k 10 200 python -u tools/regime_run.py $O/fp32_$s.npz fp32 $s
  run timeout -k 10 200 python -u tools/regime_run.py $O/fp32o_$s.npz fp32 $s --no-overlap
  run timeout -k 10 200 python -u tools/regime_run.py $O/x3split_$s.npz bf16x3 $s
  CODENERF_MEASURE=1 CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r04base.so run timeout -k 10 200 python -u tools/regime_run.py $O/x3hi_$s.npz bf16x3 $s
done
for v in in-tree dw_hinocompute dw_full5 dw_full3; do
  if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
  CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 240 python -u tools/kbench.py --precision bf16 --only dw --reps 20 > $O/kbdw_$v.json 2> $O/kbdw_$v.log
done
echo r04e done
