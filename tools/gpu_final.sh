# round-end style check: gpu tests, smoke, C2 bench (default), C3/C4/C5 bench lines, profile
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-final}
bash tools/gpu_check.sh $TAG || exit 1
for c in c3 c4 c5; do
  timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline --no-fp32 --steps 10 --warmup 3 > $O/bench_${TAG}_$c.log 2>&1 || { tail -20 $O/bench_${TAG}_$c.log; exit 1; }
  tail -1 $O/bench_${TAG}_$c.log | cut -c1-200
done
bash tools/gpu_profile.sh r02x || exit 1
