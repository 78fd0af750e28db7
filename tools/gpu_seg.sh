#!/bin/bash
# Ray-segmented march: parity tests, then per-rank times of the tile split (rank_sim)
# for the default kernel and the VR_SEG variants given as arguments.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/seg && export TMPDIR=/tmp
O=gpurun_out/seg
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "segmented or every_kernel_path" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
CAMS=${CAMS:-C0 C1}
for CAM in $CAMS; do
  timeout -k 10 200 python -u tools/rank_sim.py --camera $CAM > $O/rank_def_$CAM.log 2>&1 || exit 1
  for S in "$@"; do
    VR_PATH=7 VR_SEG=$S timeout -k 10 200 python -u tools/rank_sim.py --camera $CAM > $O/rank_s${S}_$CAM.log 2>&1 || exit 1
  done
done
for f in $O/rank_*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
