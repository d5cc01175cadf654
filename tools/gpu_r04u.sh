#!/bin/bash
# round 4 (u): 2-rank rehearsal of bench.py's N > 1 path on one GPU (gloo, both ranks on cuda:0)
export TMPDIR=/tmp OMP_NUM_THREADS=8
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --one-device > $O/dp2.log 2>&1
echo "rc=$?"
tail -1 $O/dp2.log | cut -c1-400
