#!/bin/bash
# round 6 (i): bf16x3 chains with the weight-stream pieces spread over their
# issue window (the bf16 chains keep the burst): the full GPU suite except the
# long train-PSNR files (run by gpu_j.sh), smoke, kbench A/B against r06g, bench.
export TMPDIR=/tmp
OUT=gpurun_out/r06i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_regime.py --deselect tests/test_gpu_regime_fine.py --deselect tests/test_gpu_converge.py \
  > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
for rep in 1 2; do
  for lib in base new; do
    case $lib in base) L=variants/r06g.so;; new) L=;; esac
    for prec in bf16x3f bf16x3 bf16; do
      echo "== rep $rep lib $lib prec $prec" >> $OUT/kb.log
      CODENERF_MEASURE=1 CODENERF_LIB=$L timeout -k 10 150 python tools/kbench.py --only fwd,bwd --reps 20 \
        --precision $prec >> $OUT/kb.log 2>&1 || exit 1
    done
  done
done
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
echo r06i done
