# A/B: 12-wave backward chain (tile epilogues, 3 waves per SIMD) vs default + its correctness tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash tools/gpu_variants.sh "--only fwd,bwd" base w12 base w12 > $O/var8.log 2>&1 || exit 1
CODENERF_LIB=$R/code-nerf_amd/libcodenerf_hip_w12.so timeout -k 10 500 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_dw.py tests/test_gpu_configs.py tests/test_gpu_fine.py tests/test_gpu_parity.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > $O/w12_tests.log 2>&1; echo "w12 tests rc=$?" >> $O/var8.log
