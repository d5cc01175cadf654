#!/bin/bash
# round 4 (h): one-object test, smoke, C2 bench, rocprof passes; then the
# weights-bf16 emulation variants (tools/split_emu.py, torch on the GPU)
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04h; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  tests/test_gpu_dw.py tests/test_gpu_converge.py::test_early_train_psnr_matches_reference_at_each_precision > $O/pytest_converge.log 2>&1
run timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run timeout -k 10 240 python -u tools/kbench.py --precision fp32 --only dw --reps 10 > $O/kbdw_fp32.json 2> $O/kbdw_fp32.log
cat $O/kbdw_fp32.json
run timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-300
run bash tools/gpu_profile.sh r04h/prof
EMU_DEVICE=cuda EMU_THREADS=16 EMU_ONLY=f_path,s3_dwx,wb_s2,wb_fwd,wb_bwd run timeout -k 10 420 python -u tools/split_emu.py many 320 > $O/split_emu_wb.log 2>&1
echo r04h done
