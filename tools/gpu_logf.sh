#!/bin/bash
# Table-based logf: exhaustive self-test, entropy parity tests, m3/m6 timings.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/logf; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fast_log or small_scene or codec or every_kernel or bin_counts or flex" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
for CAM in C0 C1; do for M in 3 6; do
  timeout -k 10 240 python -u bench.py --method $M --camera $CAM --no-cpu-baseline > $O/b_${CAM}_m$M.log 2>&1 || { tail $O/b_${CAM}_m$M.log; exit 1; }
  echo "$CAM m$M: $(grep -o '"kernel_ms": [0-9.]*' $O/b_${CAM}_m$M.log) $(grep -o '"value": [0-9.]*' $O/b_${CAM}_m$M.log | head -1) $(grep -o '"kernel": "[^"]*' $O/b_${CAM}_m$M.log)"
done; done
