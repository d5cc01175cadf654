#!/bin/bash
# round 5 (i): bf16x3 chain16 tile pipeline (per-tile conversions spread over the next tile) -- parity
# tests, kbench / bench A/B against the 8-wave build (libcodenerf_hip_r05w8.so)
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16x3.py tests/test_gpu_planes.py tests/test_gpu_dw.py tests/test_gpu_x3_trace.py > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" $O/pytest.log | head -60; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for rep in 1 2; do
  for lib in w8 pipe; do
    if [ $lib = w8 ]; then export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r05w8.so CODENERF_MEASURE=1; else unset CODENERF_LIB CODENERF_MEASURE; fi
    timeout -k 10 120 python -u tools/kbench.py --precision bf16x3 --only fwd,bwd > $O/kb_${lib}_$rep.log 2>&1 || { tail -20 $O/kb_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/kb_${lib}_$rep.log)"
    timeout -k 10 200 python -u bench.py --precision bf16x3 --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > $O/bench_x3_${lib}_$rep.log 2>&1 || { tail -20 $O/bench_x3_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(tail -1 $O/bench_x3_${lib}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("ms_per_step_median"))')"
  done
done
unset CODENERF_LIB CODENERF_MEASURE
bash tools/gpu_stalls.sh r05i/x3pipe bf16x3 || exit 1
echo r05i done
