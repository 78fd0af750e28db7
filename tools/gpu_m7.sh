#!/bin/bash
# Pipelined method 7: parity tests + C0/C1 timings (pipe vs plain, occupancy caps).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/m7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "small_scene or bin_counts or method7 or isabel or edge or inside or render_parameters" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
for CAM in C0 C1; do for V in "VR_M7_QUAD=0" "VR_M7_QUAD=1" "VR_M7_QUAD=1 VR_WG_PER_CU=3" "VR_M7_QUAD=1 VR_WG_PER_CU=1"; do
  env $V timeout -k 10 240 python -u bench.py --method 7 --camera $CAM --no-cpu-baseline > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  echo "$CAM $V: $(grep -o '"kernel_ms": [0-9.]*' $O/b.log) $(grep -o '"value": [0-9.]*' $O/b.log | head -1) $(grep -o '"kernel": "[^"]*' $O/b.log)"
done; done
