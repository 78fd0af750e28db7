#!/bin/bash
# k_march_wq pixel map A/B (VR_WQ_MAP=0 row per wave, 1 16x4 blocks): parity + bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
for MAP in 1; do VR_WQ_MAP=$MAP timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or random" > gpurun_out/wide/pytest_map$MAP.log 2>&1 || { tail -30 gpurun_out/wide/pytest_map$MAP.log; exit 1; }; tail -1 gpurun_out/wide/pytest_map$MAP.log; done
for A in "1024x32 C1" "1024x16 C1" "512x32 C1" "1024x32 C0"; do
  set -- $A
  for MAP in 0 1; do
    VR_WQ_MAP=$MAP timeout -k 10 300 python -u bench.py --config $1 --camera $2 --method 1 --no-cpu-baseline --steps 10 > gpurun_out/wide/map_$1_$2_$MAP.log 2>&1 || { tail -5 gpurun_out/wide/map_$1_$2_$MAP.log; exit 1; }
    echo "$1 $2 map=$MAP $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/map_$1_$2_$MAP.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/map_$1_$2_$MAP.log)"
  done
done
