#!/bin/bash
# coarse row-aligned wide-record entropy: box (default now) vs quad march (VR_BOX3=0); parity
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or isabel or coarse" > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
for B3 in 1 0; do
  for CFG in 512x32; do
    VR_BOX3=$B3 timeout -k 10 300 python -u bench.py --config $CFG --camera C0 --method 3 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wide/box3_${CFG}_$B3.log 2>&1 || { tail -5 gpurun_out/wide/box3_${CFG}_$B3.log; exit 1; }
    echo "$CFG C0 m3 VR_BOX3=$B3 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/box3_${CFG}_$B3.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/box3_${CFG}_$B3.log)"
  done
done
