#!/bin/bash
# adaptive tile order vs the estimate order (VR_NO_ADAPT), full frame, C0 / C1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/adapt && export TMPDIR=/tmp
O=gpurun_out/adapt
for cam in C0 C1; do
  timeout -k 10 240 env VR_NO_ADAPT=1 python -u bench.py --no-cpu-baseline --camera $cam --steps 40 > $O/est_$cam.log 2>&1 || { tail -20 $O/est_$cam.log; exit 1; }
  tail -1 $O/est_$cam.log
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --camera $cam --steps 40 > $O/adapt_$cam.log 2>&1 || { tail -20 $O/adapt_$cam.log; exit 1; }
  tail -1 $O/adapt_$cam.log
done
