# A/B: dual-accumulator tile chain vs default; then the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash tools/gpu_variants.sh "--only fwd,bwd" base tile2 base tile2 > $O/var7.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_r02w.log 2>&1 || { tail -20 $O/bench_r02w.log; exit 1; }
tail -1 $O/bench_r02w.log
