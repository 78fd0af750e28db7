#!/bin/bash
# round 4, job ag: entropy of mid-size row-aligned frames -- wave-staged vs LDS box vs pipe
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4ag; mkdir -p $O
for CFG in 256x4 256x8@512x512 256x2@512x512 128x1; do
  timeout -k 10 600 python -u tools/bench_variants.py --config $CFG --cameras C0,C1 --method 3 --rounds 4 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=4" "VR_PATH=7,VR_SEG=-2" > $O/v.log 2>&1 || { tail -20 $O/v.log; exit 1; }
  grep -v "round\|amdgpu.ids" $O/v.log | tee -a $O/variants_midsize_m3.log
done
echo done
