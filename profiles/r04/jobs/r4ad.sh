#!/bin/bash
# round 4, job ad: mid-size row-aligned frames (4 pixels per voxel face, 262 K rays) on the
# two/three-samples-per-box march, 2 / 4 / 8 bins, methods 1 / 2
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4ad; mkdir -p $O
for CFG in 256x4 256x8@512x512 256x2@512x512 384x4@768x768; do
  for M in 1 2; do
    timeout -k 10 600 python -u tools/bench_variants.py --config $CFG --cameras C0 --method $M --rounds 5 --env "" "VR_PATH=1,VR_DUO=2" "VR_PATH=1,VR_DUO=3" "VR_PATH=1,VR_DUO=4" > $O/v.log 2>&1 || { tail -20 $O/v.log; exit 1; }
    grep -v "round\|amdgpu.ids" $O/v.log | tee -a $O/variants_midsize_duo.log
  done
done
echo done
