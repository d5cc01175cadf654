#!/bin/bash
# round 4 (aa): LO dW bodies issue slab st + depth before slab st lands (split barrier) --
# dW / bf16x3 parity, kbench A/B against the base build (libcodenerf_hip_base.so)
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04aa; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dw.py tests/test_gpu_bf16x3.py > $O/pytest.log 2>&1 || { echo "tests failed"; grep -n "FAILED\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in in-tree base; do
    if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
    CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 240 python -u tools/kbench.py --precision bf16x3 --only dw --reps 20 > $O/kbdw_bf16x3_${v}_$rep.json 2> $O/kbdw_bf16x3_${v}_$rep.log || exit 1
    cat $O/kbdw_bf16x3_${v}_$rep.json
  done
done
for v in in-tree base; do
  if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
  CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 300 python -u bench.py --precision bf16x3 --no-cpu-baseline --no-fp32 --steps 40 > $O/b_$v.log 2>&1 || exit 1
  tail -1 $O/b_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['ms_per_step_median'])"
done
echo r04aa done
