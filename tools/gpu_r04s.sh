#!/bin/bash
# round 4 (s): dW parity; kbench A/B of the fp32 one-tile-ahead reads (r04r vs
# r04q builds) and the branch-free sigma-head MFMA (in-tree vs r04r); C5 line
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dw.py > $O/pytest_dw.log 2>&1 || { echo "dw tests failed"; grep -n "FAILED\|Error" $O/pytest_dw.log | head; exit 1; }
tail -1 $O/pytest_dw.log
for rep in 1 2; do
  for v in in-tree r04r r04q; do
    if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
    for p in bf16 fp32; do
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 240 python -u tools/kbench.py --precision $p --only dw --reps 10 > $O/kbdw_${p}_${v}_$rep.json 2> $O/kbdw_${p}_${v}_$rep.log || exit 1
      cat $O/kbdw_${p}_${v}_$rep.json
    done
  done
done
timeout -k 10 400 python -u bench.py --config c5 --no-cpu-baseline --steps 4 --warmup 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
tail -1 $O/bench_c5.log | cut -c1-200
echo r04s done
