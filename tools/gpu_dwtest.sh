set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dw.py -x -v --timeout 120 --timeout-method thread > $O/pt_dw.log 2>&1; rc=$?
tail -15 $O/pt_dw.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/kbench.py --only dw,bwd
