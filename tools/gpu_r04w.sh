#!/bin/bash
# round 4 (w): LO dW bodies with the hi / lo MFMAs of a column software-pipelined
# -- dW parity, kbench A/B against the final-tree build (libcodenerf_hip_r04t.so)
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dw.py tests/test_gpu_bf16x3.py > $O/pytest.log 2>&1 || { echo "tests failed"; grep -n "FAILED\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in in-tree r04t; do
    if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
    for p in bf16x3 bf16; do
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 240 python -u tools/kbench.py --precision $p --only dw --reps 20 > $O/kbdw_${p}_${v}_$rep.json 2> $O/kbdw_${p}_${v}_$rep.log || exit 1
      cat $O/kbdw_${p}_${v}_$rep.json
    done
  done
done
echo r04w done
