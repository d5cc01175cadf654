# A/B of the tile-epilogue chain variant + its bf16 correctness tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; cd $R
bash tools/gpu_variants.sh "--only fwd,bwd" base tile base tile > $O/var6.log 2>&1 || exit 1
CODENERF_LIB=$R/code-nerf_amd/libcodenerf_hip_tile.so timeout -k 10 400 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_configs.py tests/test_gpu_dw.py tests/test_gpu_parity.py tests/test_gpu_fine.py -x -q --timeout 120 --timeout-method thread > $O/tile_tests.log 2>&1; echo "tile tests rc=$?" >> $O/var6.log
