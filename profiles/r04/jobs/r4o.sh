#!/bin/bash
# round 4, job o: tiled plane axis copy (tests), then the final build's measurement, part 1
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_baked.py > $O/pytest_r4o.log 2>&1 || { tail -30 $O/pytest_r4o.log; exit 1; }
tail -1 $O/pytest_r4o.log
RANKSIM=0 bash tools/gpu_round.sh r05a 1024x8:C0 1024x8:C1 1024x8:S 1024x8:S:baked 512x8:C0 512x8:C0::2
