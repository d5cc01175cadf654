# A/B: two 32-sample groups per backward wave (one wave per SIMD) vs default, + bf16 correctness
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash tools/gpu_variants.sh "--only bwd" base ng2 ng2d base ng2 ng2d > $O/var13.log 2>&1 || exit 1
CODENERF_LIB=$R/code-nerf_amd/libcodenerf_hip_ng2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_dw.py tests/test_gpu_configs.py tests/test_gpu_fine.py -x -q --timeout 120 --timeout-method thread > $O/ng2_tests.log 2>&1; echo "ng2 tests rc=$?" >> $O/var13.log
