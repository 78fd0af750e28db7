#!/bin/bash
# Occupancy cap (VR_WG_PER_CU) for the codec march, methods 4/5/6 at C0.
# usage: bash tools/gpu_occ_codec.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/occc && export TMPDIR=/tmp
for M in 4 5 6; do
  for W in 0 1 2 3 4 6; do
    if [ $W -gt 0 ]; then export VR_WG_PER_CU=$W; else unset VR_WG_PER_CU; fi
    timeout -k 10 240 python -u bench.py --method $M --no-cpu-baseline > gpurun_out/occc/m${M}_w$W.log 2>&1 || exit $?
    echo "m$M wg=$W: $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/occc/m${M}_w$W.log) $(grep -o '"value": [0-9.]*' gpurun_out/occc/m${M}_w$W.log | head -1)"
  done
done
