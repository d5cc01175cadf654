#!/bin/bash
# round 4 (b): the X-split / staggered-DMA / fp32-layout build: parity tests,
# kernel A/B against the round-start library, trained vs random-init weights,
# effective clocks of the forward chain (kbench vs bench).
export TMPDIR=/tmp OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
O=gpurun_out/r04b; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
run timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_dw.py tests/test_gpu_planes.py tests/test_gpu_bf16x3.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
for p in bf16 bf16x3 fp32; do
  for lib in base new; do
    if [ $lib = base ]; then L=$PWD/code-nerf_amd/libcodenerf_hip_r04base.so; else L=; fi
    CODENERF_MEASURE=1 CODENERF_LIB=$L run timeout -k 10 240 python -u tools/kbench.py --precision $p --only fwd,bwd,dw --reps 20 > $O/kb_${p}_${lib}.json 2> $O/kb_${p}_${lib}.log
  done
done
run timeout -k 10 400 python -u tools/make_bench_weights.py 400 8 > $O/mkw.log 2>&1
cp weights/c2_regime_400.pth $O/
for w in none weights/c2_regime_400.pth; do
  for p in bf16 bf16x3; do
    run timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32 --steps 30 --warmup 10 --precision $p --weights $w > $O/bench_${p}_$(basename $w).json 2> $O/bench_${p}_$(basename $w).log
  done
done
R=$PWD
cd /tmp
run timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $R/$O/clk_kbench -o run --output-format csv -- python3 $R/tools/kbench.py --only fwd --reps 5 > $R/$O/clk_kbench.log 2>&1
for w in none weights/c2_regime_400.pth; do
  run timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $R/$O/clk_bench_$(basename $w) -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-fp32 --steps 10 --warmup 5 --weights $w > $R/$O/clk_bench_$(basename $w).log 2>&1
done
echo r04b done
