# finer stall counters of the chain kernels (kbench fwd/bwd launches alone), two passes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/st1 $O/st2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE --output-format csv -d $O/st1 -- python3 $R/tools/kbench.py --only fwd,bwd --reps 3 > $O/st1.log 2>&1 || { tail -5 $O/st1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/st2 -- python3 $R/tools/kbench.py --only fwd,bwd --reps 3 > $O/st2.log 2>&1 || { tail -5 $O/st2.log; exit 1; }
echo stall2 ok
