#!/bin/bash
# round 4, job u: consecutive frames on two alternating streams (ramp / tail overlap)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4u; mkdir -p $O
for CAM in C0 C1 S; do
  timeout -k 10 400 python -u tools/overlap_sim.py --camera $CAM --worlds 1,2,4,8 > $O/overlap_$CAM.log 2>&1 || { tail -20 $O/overlap_$CAM.log; exit 1; }
  grep -v amdgpu.ids $O/overlap_$CAM.log
done
timeout -k 10 400 python -u tools/overlap_sim.py --config 512x8 --camera C0 --worlds 1,4,8 > $O/overlap_512_C0.log 2>&1 || exit 1
grep -v amdgpu.ids $O/overlap_512_C0.log
echo done
