#!/bin/bash
# ADVICE r01 fixes: new occupancy-cap parity cases, codec occupancy sweep (now applied).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r02a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "every_kernel_path or codec or method7 or small_scene" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_occ_codec.sh > $O/occupancy_codec.log 2>&1 || { tail $O/occupancy_codec.log; exit 1; }
cat $O/occupancy_codec.log
