#!/bin/bash
# round 4, job af: oblique coarse frames on the K-samples box march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4af; mkdir -p $O
for CFG in 512x8 256x4; do
  for M in 1 2; do
    timeout -k 10 600 python -u tools/bench_variants.py --config $CFG --cameras C1 --method $M --rounds 4 --env "" "VR_PATH=1,VR_DUO=0" "VR_PATH=1,VR_DUO=2" "VR_PATH=1,VR_DUO=4" > $O/v.log 2>&1 || { tail -20 $O/v.log; exit 1; }
    grep -v "round\|amdgpu.ids" $O/v.log | tee -a $O/variants_oblique_duo.log
  done
done
echo done
