#!/bin/bash
# round 5 (m): (1) timing-only chain16 probes (no barrier / no weight stream,
# results invalid); (2) bf16x3 on the 32-sample chains (libcodenerf_hip_x3c32.so):
# the PSNR-trajectory tests that chain16 was not run against, kbench / bench
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
for rep in 1 2; do
  for lib in default x3nobar x3nodma x3c32; do
    if [ $lib = default ]; then unset CODENERF_LIB CODENERF_MEASURE; else export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_$lib.so CODENERF_MEASURE=1; fi
    timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --only fwd,bwd > $O/kb_${lib}_$rep.log 2>&1 || { tail -20 $O/kb_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/kb_${lib}_$rep.log)"
  done
done
export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_x3c32.so CODENERF_MEASURE=1
timeout -k 10 200 python -u bench.py --precision bf16x3 --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > $O/bench_x3c32.log 2>&1 || { tail -20 $O/bench_x3c32.log; exit 1; }
echo "x3c32 bench: $(tail -1 $O/bench_x3c32.log | cut -c1-200)"
timeout -k 10 900 python -u -m pytest -v -s --timeout 850 --timeout-method thread tests/test_gpu_bf16x3.py \
  "tests/test_gpu_regime_fine.py::test_fine_regime_long_horizon_vs_reference" \
  "tests/test_gpu_converge.py::test_early_train_psnr_matches_reference_at_each_precision" \
  tests/test_gpu_x3_trace.py "tests/test_gpu_regime.py::test_seed3_bf16x3_exit_is_its_arithmetic" > $O/pytest_x3c32.log 2>&1; rc=$?
grep -E "PASS|FAIL|horizon|replayable|ratio  [2-9]|first epoch|assert" $O/pytest_x3c32.log | cut -c1-300 | head -40; ok $rc || exit $rc
echo r05m done
