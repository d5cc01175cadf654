#!/bin/bash
# round 4 (n): launch-recorded timers, last dW on the main stream, coalesced
# latent_fwd, finer dw_fold, fp32 dW byte fallback -- parity subset, smoke,
# bench, step timeline
set -o pipefail
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_dw.py tests/test_gpu_fine.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_train.py > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -n "FAILED\|Error" $O/pytest.log | head; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
bash tools/gpu_profile.sh r04n/prof || exit 1
echo r04n done
