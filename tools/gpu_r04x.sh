#!/bin/bash
# round 4 (x): five more seeds of the many-object long-horizon PSNR measurement
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 1100 python -u tools/regime_seeds.py $O/seeds.json 3 4 5 6 7 > $O/seeds.log 2>&1
echo "rc=$?"
grep '"seed"' $O/seeds.log | cut -c1-300
