# rocprofv3 kernel stats + HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) of bench.py
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; TAG=${1:-prof}; mkdir -p $O
B="$R/bench.py --steps 10 --warmup 3 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
rm -rf $O/${TAG}_stats $O/${TAG}_fetch $O/${TAG}_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_stats -- python3 $B > $O/${TAG}_stats.log 2>&1 || { tail -20 $O/${TAG}_stats.log; exit 1; }
tail -1 $O/${TAG}_stats.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetch -- python3 $B > $O/${TAG}_fetch.log 2>&1 || { tail -20 $O/${TAG}_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_write -- python3 $B > $O/${TAG}_write.log 2>&1 || { tail -20 $O/${TAG}_write.log; exit 1; }
echo profiled
