#!/bin/bash
# round 5 (p): bf16x3 dX chain with counted mask reads (kAsmLds backward) --
# bf16x3 parity / trajectory tests, kbench / bench A/B against libcodenerf_hip_r05base.so
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16x3.py tests/test_gpu_planes.py tests/test_gpu_dw.py tests/test_gpu_x3_trace.py > $O/pytest.log 2>&1; rc=$?
grep -cE "PASSED" $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for rep in 1 2; do
  for lib in base cntm; do
    if [ $lib = base ]; then export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r05base.so CODENERF_MEASURE=1; else unset CODENERF_LIB CODENERF_MEASURE; fi
    timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --only fwd,bwd > $O/kb_${lib}_$rep.log 2>&1 || { tail -20 $O/kb_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/kb_${lib}_$rep.log)"
    timeout -k 10 200 python -u bench.py --precision bf16x3 --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > $O/bench_${lib}_$rep.log 2>&1 || { tail -20 $O/bench_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/bench_${lib}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("ms_per_step_median"))')"
  done
done
unset CODENERF_LIB CODENERF_MEASURE
timeout -k 10 900 python -u -m pytest -v -s --timeout 850 --timeout-method thread \
  "tests/test_gpu_regime_fine.py::test_fine_regime_long_horizon_vs_reference" \
  "tests/test_gpu_converge.py::test_early_train_psnr_matches_reference_at_each_precision" \
  "tests/test_gpu_regime.py::test_seed3_bf16x3_exit_is_its_arithmetic" > $O/pytest_traj.log 2>&1; rc=$?
grep -E "PASSED|FAILED|first epoch|replayable prefix \(within" $O/pytest_traj.log | cut -c1-250 | head; ok $rc || exit $rc
echo r05p done
