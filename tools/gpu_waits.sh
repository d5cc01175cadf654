#!/bin/bash
# Stall breakdown of the hot kernels (tools/kbench.py launches each alone):
#   tools/gpu_waits.sh <tag> [kbench args]
# Two PMC passes (8 SQ counters each + GRBM); every step time-limited.
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KB="tools/kbench.py --reps 5 $*"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS -d "$OUT/waits" -o run --output-format csv -- python3 $KB > "$OUT/waits.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d "$OUT/cyc" -o run --output-format csv -- python3 $KB > "$OUT/cyc.log" 2>&1 || exit $?
echo "waits $TAG done"
