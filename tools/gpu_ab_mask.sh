set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash tools/gpu_variants.sh "--only fwd,bwd" base pk mask base pk mask > $O/var3.log 2>&1 || exit 1
# correctness of the mask variant on the bf16 chain: planes + C2 train step
CODENERF_LIB=$R/code-nerf_amd/libcodenerf_hip_mask.so timeout -k 10 300 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/mask_tests.log 2>&1; echo "mask tests rc=$?" >> $O/var3.log
