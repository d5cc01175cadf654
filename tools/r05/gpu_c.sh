#!/bin/bash
# round 5 (c): first run of the 16x16x32 bf16x3 chains (chain16.hip): parity tests, kernel timings, a bench line
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bf16x3.py tests/test_gpu_planes.py "tests/test_gpu_dw.py" -k "x3 or bf16x3" > $O/pytest_x3.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|rgb max" $O/pytest_x3.log | head -40
[ $rc -eq 0 ] || { tail -60 $O/pytest_x3.log; exit $rc; }
timeout -k 10 200 python -u tools/kbench.py --precision bf16x3 --only fwd,bwd,dw > $O/kbench_x3.log 2>&1 || { tail -30 $O/kbench_x3.log; exit 1; }
cat $O/kbench_x3.log | tail -8
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 1500 $O/bench.log
echo r05c done
