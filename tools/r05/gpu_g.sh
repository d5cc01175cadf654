#!/bin/bash
# round 5 (g): dW LO tile ring (DwLo) -- parity tests + kbench A/B against the
# pre-change library (libcodenerf_hip_r05old.so); the new bf16x3 tests
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dw.py tests/test_gpu_bf16x3.py > $O/pytest_dw.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" $O/pytest_dw.log | head -30; [ $rc -eq 0 ] || { tail -40 $O/pytest_dw.log; exit $rc; }
for rep in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r05old.so CODENERF_MEASURE=1; else unset CODENERF_LIB CODENERF_MEASURE; fi
    timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --only dw > $O/kb_dw_${lib}_$rep.log 2>&1 || { tail -20 $O/kb_dw_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/kb_dw_${lib}_$rep.log)"
  done
done
unset CODENERF_LIB CODENERF_MEASURE
for rep in 1 2; do
  for lib in old new; do
    if [ $lib = old ]; then export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r05old.so CODENERF_MEASURE=1; else unset CODENERF_LIB CODENERF_MEASURE; fi
    timeout -k 10 200 python -u bench.py --precision bf16x3 --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > $O/bench_x3_${lib}_$rep.log 2>&1 || { tail -20 $O/bench_x3_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/bench_x3_${lib}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("ms_per_step_median"))')"
  done
done
unset CODENERF_LIB CODENERF_MEASURE
timeout -k 10 900 python -u -m pytest -v -s --timeout 850 --timeout-method thread tests/test_gpu_x3_trace.py \
  "tests/test_gpu_regime.py::test_seed3_bf16x3_exit_is_its_arithmetic" \
  "tests/test_gpu_configs.py::test_module_forward_over_budget_recomputes_parts" > $O/pytest_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|ratio|first epoch|assert" $O/pytest_new.log | cut -c1-300 | head -50; ok $rc || exit $rc
echo r05g done
