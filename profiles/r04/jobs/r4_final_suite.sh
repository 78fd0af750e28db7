#!/bin/bash
# round 4 final build: the whole -m gpu suite + smoke (what the driver runs), then the rank
# simulation with the N > 1 frame loop's measured host cost added (0.017 ms per frame,
# profiles/r04/host_cost_N8_r4h.log: ring-8 period 0.2150 vs renders alone 0.1984)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_suite.sh r4suite || exit 1
O=gpurun_out/r4suite
for CAM in C0 C1 S; do
  timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM --worlds 2,4,8 --modes cost --host-ms ${HOSTMS:-0.017} > $O/rank_sim_$CAM.log 2>&1 || exit 1
done
echo done
