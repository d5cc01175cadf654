#!/bin/bash
# Stall / issue counters of the chain kernels (tools/kbench.py launches, each
# kernel alone at C2 size), two --pmc passes (8 SQ + GRBM counters each), and
# their per-kernel summary (tools/stall_summary.py).
#   bash tools/gpu_stalls.sh TAG PRECISION [CODENERF_LIB]      (env KB_ONLY: kbench phases, default fwd,bwd)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
TAG=$1; PREC=$2; export CODENERF_LIB=${3:-} CODENERF_MEASURE=1
rm -rf $O/${TAG}_s1 $O/${TAG}_s2
KB="$R/tools/kbench.py --only ${KB_ONLY:-fwd,bwd} --reps 3 --precision $PREC"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d $O/${TAG}_s1 -- python3 $KB > $O/${TAG}_s1.log 2>&1 || { tail -5 $O/${TAG}_s1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/${TAG}_s2 -- python3 $KB > $O/${TAG}_s2.log 2>&1 || { tail -5 $O/${TAG}_s2.log; exit 1; }
cd $R && python3 tools/stall_summary.py $O/${TAG}_s1 $O/${TAG}_s2 > $O/${TAG}_stalls.md && cat $O/${TAG}_stalls.md
