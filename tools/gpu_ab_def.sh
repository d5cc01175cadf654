# A/B: tile epilogues (whole / interleaved halves) vs default
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash tools/gpu_variants.sh "--only fwd,bwd" base def0 def6 tile6 base def0 def6 tile6 > $O/var10.log 2>&1 || exit 1
