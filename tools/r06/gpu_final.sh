#!/bin/bash
# round 6 (final): the whole GPU suite in one process, as the driver runs it.
export TMPDIR=/tmp
OUT=gpurun_out/r06final
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 1000 --timeout-method thread > $OUT/pytest_all.log 2>&1
rc=$?
echo "pytest rc=$rc"
exit $rc
