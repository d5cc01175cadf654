#!/bin/bash
# round 4 (a): per-layer dW-split emulation; random-init vs trained weights;
# effective clock of the forward chain in kbench vs the bench step
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*" >&2; exit $rc; fi; }
L=$(python3 -c "
import importlib.util
s=importlib.util.spec_from_file_location('m','tools/split_emu.py'); m=importlib.util.module_from_spec(s); s.loader.exec_module(m)
print(','.join(k for k in m.VARIANTS if k.startswith(('s3_dwx_', 's3_dwdy_', 'dwx_'))))")
EMU_DEVICE=cuda EMU_ONLY=f_path,s3_dwx,$L run timeout -k 10 900 python -u tools/split_emu.py many 320 > $O/emu_layers.log 2>&1
run timeout -k 10 400 python -u tools/make_bench_weights.py 400 8 > $O/mkw.log 2>&1
cp weights/c2_regime_400.pth $O/
for w in none weights/c2_regime_400.pth; do
  for p in bf16 bf16x3; do
    run timeout -k 10 300 python bench.py --no-cpu-baseline --no-fp32 --steps 30 --warmup 10 --precision $p --weights $w > $O/bench_${p}_$(basename $w).json 2> $O/bench_${p}_$(basename $w).log
  done
done
cd /tmp
run timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $GRAFT_REPO_ROOT/$O/clk_kbench -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --only fwd --reps 5 > $GRAFT_REPO_ROOT/$O/clk_kbench.log 2>&1
for w in none weights/c2_regime_400.pth; do
  run timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $GRAFT_REPO_ROOT/$O/clk_bench_$(basename $w) -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-fp32 --steps 10 --warmup 5 --weights $w > $GRAFT_REPO_ROOT/$O/clk_bench_$(basename $w).log 2>&1
done
echo r04a done
