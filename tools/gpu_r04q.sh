#!/bin/bash
# round 4 (q): latent_fwd back to its original order, dW X fragments read one
# tile ahead -- full gpu suite; dW kbench A/B against the dW without the
# prefetch (libcodenerf_hip_dwnopf.so); bench; profile
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04q; mkdir -p $O
for rep in 1 2; do
  for v in in-tree dwnopf; do
    if [ $v = in-tree ]; then L=; else L=$PWD/code-nerf_amd/libcodenerf_hip_$v.so; fi
    for p in bf16 bf16x3; do
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 240 python -u tools/kbench.py --precision $p --only dw --reps 20 > $O/kbdw_${p}_${v}_$rep.json 2> $O/kbdw_${p}_${v}_$rep.log || exit 1
      cat $O/kbdw_${p}_${v}_$rep.json
    done
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -n "FAILED\|Error" $O/pytest_gpu.log | head; }
grep -n "passed\|failed" $O/pytest_gpu.log | tail -2
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
bash tools/gpu_profile.sh r04q/prof || exit 1
echo r04q done
