# bench.py lines for the other BASELINE configs (C3 geometry, C4 optimize, C5 fp32 256^2)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-cfg}
for c in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_${TAG}_$c.log 2>&1 || { echo "bench $c failed"; tail -20 $O/bench_${TAG}_$c.log; exit 1; }
  tail -1 $O/bench_${TAG}_$c.log
done
