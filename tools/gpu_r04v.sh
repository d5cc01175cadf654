#!/bin/bash
# round 4 (v): dX || dW overlap vs one dX and one dW launch per step, interleaved A/B, bf16 and bf16x3
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04v; mkdir -p $O
for rep in 1 2; do
  for p in bf16 bf16x3; do
    for v in overlap serial; do
      F=""; [ $v = serial ] && F="--no-overlap"
      timeout -k 10 300 python -u bench.py --precision $p --no-cpu-baseline --no-fp32 --steps 50 --warmup 10 $F > $O/b_${p}_${v}_$rep.log 2>&1 || { tail -5 $O/b_${p}_${v}_$rep.log; exit 1; }
      tail -1 $O/b_${p}_${v}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p $v $rep', d['ms_per_step'], d['ms_per_step_median'])"
    done
  done
done
echo r04v done
