#!/bin/bash
# round 4 (c): 8-B plane-store build: parity tests, chain A/B against the
# staggered-DMA build (r04s), dW LO variants, fp32 dW stall counters.
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04c; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_planes.py tests/test_gpu_dw.py tests/test_gpu_bf16x3.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
for rep in 1 2; do
for p in bf16 bf16x3; do
  for lib in r04s new; do
    if [ $lib = new ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$lib.so; fi
    CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 240 python -u tools/kbench.py --precision $p --only fwd,bwd --reps 20 > $O/kb_${p}_${lib}_$rep.json 2> $O/kb_${p}_${lib}_$rep.log
  done
done
done
for v in new dwlo_nolomma dwlo_nocompute; do
  if [ $v = new ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
  CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 240 python -u tools/kbench.py --precision bf16x3 --only dw --reps 20 > $O/kbdw_$v.json 2> $O/kbdw_$v.log
done
KB_ONLY=dw run timeout -k 10 400 bash tools/gpu_stalls.sh r04c_fp32dw fp32 > $O/stalls_fp32dw.log 2>&1
echo r04c done
