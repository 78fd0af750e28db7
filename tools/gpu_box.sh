#!/bin/bash
# LDS-box march with quad-cooperative wide-record loads: parity, then box vs default bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or isabel or coarse or every_kernel" > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
for A in "512x32 C0 -" "1024x32 C0 1" "1024x32 C0 -" "1024x16 C0 1" "1024x16 C0 -" "1024x32 C1 1" "512x32 C1 1"; do
  set -- $A
  for M in 1 3; do
    if [ "$3" = "1" ]; then export VR_PATH=1; else unset VR_PATH; fi
    timeout -k 10 300 python -u bench.py --config $1 --camera $2 --method $M --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wide/box_$1_$2_$3_m$M.log 2>&1 || { tail -5 gpurun_out/wide/box_$1_$2_$3_m$M.log; exit 1; }
    echo "$1 $2 path=$3 m$M $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/box_$1_$2_$3_m$M.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/box_$1_$2_$3_m$M.log)"
  done
done
