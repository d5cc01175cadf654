# gpu tests (all) then per-kernel timings
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt_quick.log 2>&1; rc=$?
tail -4 $O/pt_quick.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" $O/pt_quick.log | head -60; exit $rc; }
timeout -k 10 120 python -u tools/kbench.py --only fwd,bwd,dw
