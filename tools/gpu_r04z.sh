#!/bin/bash
# round 4 (z): dX / dW pipeline depth (row ranges 2 / 3 / 4), bf16 and bf16x3, interleaved
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04z; mkdir -p $O
for rep in 1 2; do
  for p in bf16x3 bf16; do
    for k in 2 3 4; do
      timeout -k 10 300 python -u bench.py --precision $p --no-cpu-baseline --no-fp32 --steps 40 --warmup 10 --bwd-ranges $k > $O/b_${p}_${k}_$rep.log 2>&1 || { tail -5 $O/b_${p}_${k}_$rep.log; exit 1; }
      tail -1 $O/b_${p}_${k}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p ranges $k rep $rep', d['ms_per_step'], d['ms_per_step_median'])"
    done
  done
done
echo r04z done
