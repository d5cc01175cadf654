#!/bin/bash
# round 6 (a): the bf16x3f plan (bf16x3 forward, bf16 backward) -- its parity
# tests, C2 fp32-class rgb at the north-star bar, the C4 fp32 slice pin, the
# clock probe; then the bench line (every precision, rooflines, clock).
export TMPDIR=/tmp
OUT=gpurun_out/r06a
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_bf16x3f.py "tests/test_gpu_configs.py::test_c2_fp32_class_rgb" \
  "tests/test_gpu_configs.py::test_c4_full_size_50_views_properties_and_ray_subset" \
  tests/test_gpu_launch_hooks.py > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
echo r06a done
