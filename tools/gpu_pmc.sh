# usage: bash tools/gpu_pmc.sh TAG "kbench args" "COUNTERS..."  -> gpurun_out/pmc_TAG (csv)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; TAG=$1; ARGS=$2; shift 2
mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/pmc_$TAG
timeout -s KILL 90 rocprofv3 --pmc $@ --output-format csv -d $O/pmc_$TAG -- python3 $R/tools/kbench.py $ARGS --reps 3 > $O/pmc_$TAG.log 2>&1 || { tail -5 $O/pmc_$TAG.log; exit 1; }
echo ok $TAG
