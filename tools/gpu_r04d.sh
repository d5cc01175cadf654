#!/bin/bash
# round 4 (d): train-PSNR regime tests on the X-split build (verdict r3 items 1, 2)
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread $@ > $O/pytest_$(echo $@ | md5sum | cut -c1-6).log 2>&1
echo "rc=$?"
