#!/bin/bash
# Measurement-only library variant (tools/kbench.py A/B, loaded with
# CODENERF_MEASURE=1 CODENERF_LIB=variants/<name>/libcodenerf_hip.so):
#   tools/r06/make_variant.sh <name> <python file patching variants/<name>/csrc> <objects to rebuild...>
# Copies code-nerf_amd/csrc with its build objects, applies the patch, marks
# every object up to date except the named ones (the patch must only change
# those kernels), and links.
set -e
N=$1; PATCH=$2; shift 2
V=variants/$N
rm -rf $V && mkdir -p $V && ln -sfn ../include variants/include
cp -rp code-nerf_amd/csrc $V/csrc
python3 $PATCH $V/csrc
find $V/csrc/build -name '*.o' -exec touch {} +
for o in "$@"; do rm -f $V/csrc/build/$o; done
make -C $V/csrc -j8 > $V/build.log 2>&1
ls -la $V/libcodenerf_hip.so
