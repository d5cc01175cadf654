# usage: bash tools/gpu_variants.sh "<kbench args>" v1 v2 ...   (variant names; "base" = default lib)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ARGS=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/code-nerf_amd/libcodenerf_hip.so; else L=$R/code-nerf_amd/libcodenerf_hip_$v.so; fi
  echo -n "$v: "
  CODENERF_LIB=$L timeout -k 10 120 python -u tools/kbench.py $ARGS 2>>$O/variants.err || { echo "FAILED $v"; tail -20 $O/variants.err; exit 1; }
done
