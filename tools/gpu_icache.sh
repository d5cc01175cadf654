# instruction-cache counters of the chain kernels (kbench fwd/bwd launches alone)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/ic1 $O/ic2
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $O/ic1 -- python3 $R/tools/kbench.py --only fwd,bwd --reps 3 > $O/ic1.log 2>&1 || { tail -5 $O/ic1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $O/ic2 -- python3 $R/tools/kbench.py --only fwd,bwd --reps 3 > $O/ic2.log 2>&1 || { tail -5 $O/ic2.log; exit 1; }
echo icache ok
