#!/bin/bash
# Occupancy cap (VR_WG_PER_CU: workgroups per CU through an LDS request) per
# kernel: full frames for methods 1/2/3/7 at C0 and C1, and the cost-dealt
# rank lists (ray-segmented march) at C0.  usage: bash tools/gpu_occ.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/occ && export TMPDIR=/tmp
for M in ${OCC_METHODS:-1 2 7}; do
  timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --rounds 3 --method $M \
    --env "" "VR_WG_PER_CU=1" "VR_WG_PER_CU=2" "VR_WG_PER_CU=3" "VR_WG_PER_CU=4" > gpurun_out/occ/m$M.log 2>&1 || exit $?
  grep -E "median" gpurun_out/occ/m$M.log | sed "s/^/m$M /"
done
for W in 0 2 3 4; do
  if [ $W -gt 0 ]; then export VR_WG_PER_CU=$W; fi
  timeout -k 10 300 python -u tools/rank_sim.py --camera C0 > gpurun_out/occ/ranks_w$W.log 2>&1 || exit $?
  echo "ranks wg=$W:"; grep "cost N=" gpurun_out/occ/ranks_w$W.log
done
