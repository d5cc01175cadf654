#!/bin/bash
# round 5 (r): 2-rank rehearsal of bench.py's N > 1 path on one GPU (gloo, both ranks on cuda:0)
export TMPDIR=/tmp OMP_NUM_THREADS=8
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --one-device > $O/dp2.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
tail -1 $O/dp2.log | cut -c1-400
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_dp.py > $O/pytest_dp.log 2>&1; echo "dp tests rc=$?"; grep -E "passed|failed" $O/pytest_dp.log | tail -1
