#!/bin/bash
# round 5 (k): static priority for waves 4-7 (s_setprio 1) in the 8-wave bf16
# and bf16x3 chains -- kbench / bench A/B against libcodenerf_hip_r05cnt.so
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_planes.py tests/test_gpu_bf16x3.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for rep in 1 2; do
  for lib in base prio; do
    if [ $lib = base ]; then export CODENERF_LIB=$PWD/code-nerf_amd/libcodenerf_hip_r05cnt.so CODENERF_MEASURE=1; else unset CODENERF_LIB CODENERF_MEASURE; fi
    for prec in bf16 bf16x3; do
      timeout -k 10 120 python -u tools/kbench.py --precision $prec --only fwd,bwd > $O/kb_${prec}_${lib}_$rep.log 2>&1 || { tail -20 $O/kb_${prec}_${lib}_$rep.log; exit 1; }
      echo "$prec $lib $rep: $(tail -1 $O/kb_${prec}_${lib}_$rep.log)"
      timeout -k 10 200 python -u bench.py --precision $prec --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > $O/bench_${prec}_${lib}_$rep.log 2>&1 || { tail -20 $O/bench_${prec}_${lib}_$rep.log; exit 1; }
      echo "$prec $lib $rep: $(tail -1 $O/bench_${prec}_${lib}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("ms_per_step_median"))')"
    done
  done
done
echo r05k done
