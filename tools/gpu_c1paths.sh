#!/bin/bash
# C1 (oblique) kernel-path comparison: quad (default) vs per-ray pipelined vs
# ray-segmented, bench's HIP-event kernel ms.  usage: bash tools/gpu_c1paths.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c1p && export TMPDIR=/tmp
for P in 0 2 7; do
  VR_PATH=$P timeout -k 10 240 python -u bench.py --camera C1 --no-cpu-baseline > gpurun_out/c1p/path$P.log 2>&1 || exit $?
  echo "path $P: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/c1p/path$P.log) $(grep -o '"value": [0-9.]*' gpurun_out/c1p/path$P.log)"
done
