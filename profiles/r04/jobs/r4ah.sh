#!/bin/bash
# round 4, job ah: small-frame entropy dispatch -- GPU suite, then configs 1/2 entropy timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_suite.sh r4ah || exit 1
O=gpurun_out/r4ah
for CFG in 256x4 128x1; do
  timeout -k 10 600 python -u tools/bench_variants.py --config $CFG --cameras C0,C1 --method 3 --rounds 4 --env "" "VR_PATH=4" "VR_PATH=2" > $O/v.log 2>&1 || { tail -20 $O/v.log; exit 1; }
  grep -v "round\|amdgpu.ids" $O/v.log | tee -a $O/variants_small_m3.log
done
echo done
