#!/bin/bash
# parity of the segmented variants + rank_sim with the default kernel choice (m1, m2)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/segdef && export TMPDIR=/tmp
O=gpurun_out/segdef
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "seg or every_kernel or bench or tile" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in 1 2; do
  timeout -k 10 200 python -u tools/rank_sim.py --method $m > $O/rank_m$m.log 2>&1 || { cat $O/rank_m$m.log; exit 1; }
  echo "== m$m"; grep -v amdgpu.ids $O/rank_m$m.log | grep -v "tiles alone"
done
