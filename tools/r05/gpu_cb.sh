#!/bin/bash
# c (chain16 first run) then b (trace + seed-3 emulation) unless c ended in a fault / timeout
bash tools/r05/gpu_c.sh; rc=$?
echo "gpu_c rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then bash tools/r05/gpu_b.sh; else exit $rc; fi
