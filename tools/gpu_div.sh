#!/bin/bash
# exact reciprocal division in the codec decode: self-test + codec/wide parity, codec bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_baked.py tests/test_gpu_io.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
for CFG in 1024x32 1024x8; do
  for CAM in C0 C1; do
    for M in 4 5 6; do
      timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method $M --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wide/${CFG}_${CAM}_m$M.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_${CAM}_m$M.log; exit 1; }
      echo "$CFG $CAM m$M $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m$M.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_${CAM}_m$M.log)"
    done
  done
done
