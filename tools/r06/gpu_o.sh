#!/bin/bash
# round 6 (o, final kernels): profiles of the C2 step in bf16x3f (the headline), bf16x3 and
# bf16 (kernel stats, MFMA busy, FETCH_SIZE, WRITE_SIZE passes) -- summarised
# locally by tools/prof_summary.py into profiles/r06o_*_kernels.md and
# profiles/pmc_traffic.json -- and the bench line of this tree.
export TMPDIR=/tmp
bash tools/gpu_profile.sh r06o/x3f --precision bf16x3f || exit 1
bash tools/gpu_profile.sh r06o/x3 --precision bf16x3 || exit 1
bash tools/gpu_profile.sh r06o/b16 --precision bf16 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r06o/bench.log 2>&1 || exit 1
echo r06o done
