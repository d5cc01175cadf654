#!/bin/bash
# round 5 (f): the trace against the kernel-faithful emulation (OPS_BF16X3_K:
# three-product splits, the encoding_shape fold); seed-3 emulation
# trajectories; the new / changed GPU tests; chain stall counters
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 300 python -u tools/x3_trace.py $O/trace_seed3_k.json 3 96 104 > $O/trace_seed3_k.log 2>&1; rc=$?
grep -A32 "step 104" $O/trace_seed3_k.log | head -34; ok $rc || exit $rc
EMU_DEVICE=cuda EMU_THREADS=16 EMU_ONLY=x3_k,x3_kernel,f_path timeout -k 10 600 python -u tools/split_emu.py many 320 3 > $O/emu_seed3.log 2>&1; rc=$?
grep "epoch-mean" $O/emu_seed3.log | cut -c1-300; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  "tests/test_gpu_converge.py::test_early_train_psnr_matches_reference_at_each_precision" \
  "tests/test_gpu_regime_fine.py::test_fine_regime_c2_image_size_vs_reference" \
  "tests/test_gpu_configs.py::test_module_forward_over_budget_recomputes_parts" > $O/pytest_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|horizon|replayable|assert" $O/pytest_new.log | cut -c1-400 | head -40; ok $rc || exit $rc
bash tools/gpu_stalls.sh r05f/x3 bf16x3 || exit 1
bash tools/gpu_stalls.sh r05f/b16 bf16 || exit 1
echo r05f done
