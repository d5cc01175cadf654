#!/bin/bash
# round 4 (i): batched dW staging for the small bf16 bodies -- dW parity,
# kbench A/B against the HEAD dW (libcodenerf_hip_dwbase.so), C2 step; then
# the PSNR regime tests with their printed gaps
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04i; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dw.py > $O/pytest_dw.log 2>&1
tail -1 $O/pytest_dw.log
for rep in 1 2; do
  for v in in-tree dwbase; do
    if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
    CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 240 python -u tools/kbench.py --precision bf16 --only dw --reps 20 > $O/kbdw_${v}_$rep.json 2> $O/kbdw_${v}_$rep.log
    cat $O/kbdw_${v}_$rep.json
  done
done
for v in in-tree dwbase; do
  if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
  CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-fp32 --steps 30 > $O/bench_$v.log 2>&1
  tail -1 $O/bench_$v.log | cut -c1-260
done
run timeout -k 10 900 python -u -m pytest -x -v -s --timeout 850 --timeout-method thread tests/test_gpu_regime.py tests/test_gpu_regime_fine.py > $O/pytest_regime.log 2>&1
tail -1 $O/pytest_regime.log
echo r04i done
