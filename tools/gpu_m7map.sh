#!/bin/bash
# k_march_m7wq pixel map A/B: parity under the new default, bench lines map 0 / 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or random" > gpurun_out/wide/pytest_m7map.log 2>&1 || { tail -30 gpurun_out/wide/pytest_m7map.log; exit 1; }
tail -1 gpurun_out/wide/pytest_m7map.log
for A in "1024x32 C1" "1024x32 C0" "1024x16 C1"; do
  set -- $A
  for MAP in 0 1; do
    VR_WQ_MAP=$MAP timeout -k 10 300 python -u bench.py --config $1 --camera $2 --method 7 --no-cpu-baseline --steps 10 > gpurun_out/wide/m7map_$1_$2_$MAP.log 2>&1 || { tail -5 gpurun_out/wide/m7map_$1_$2_$MAP.log; exit 1; }
    echo "$1 $2 m7 map=$MAP $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/m7map_$1_$2_$MAP.log)"
  done
done
