#!/bin/bash
# Sweep the XCD block shape of the full-frame order (VR_XBLOCK=bx,by tiles of
# 64x4 px per block dealt to one XCD) at C0 and C1: bench kernel ms + Mrays/s.
# usage: bash tools/gpu_xblock.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/xb && export TMPDIR=/tmp
for CAM in C0 C1; do
  for XB in 1,4 1,1 1,2 1,8 1,16 2,4 2,8 4,4 4,16 1,32; do
    VR_XBLOCK=$XB timeout -k 10 240 python -u bench.py --camera $CAM --no-cpu-baseline > gpurun_out/xb/${CAM}_$XB.log 2>&1 || exit $?
    echo "$CAM xblock $XB: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/xb/${CAM}_$XB.log) $(grep -o '"value": [0-9.]*' gpurun_out/xb/${CAM}_$XB.log)"
  done
done
