#!/bin/bash
# rank_sim over cameras/methods for the default kernels and seg variants
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/seg2 && export TMPDIR=/tmp
O=gpurun_out/seg2
run() { # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/rank_sim.py $ARGS > $O/$tag.log 2>&1 || { cat $O/$tag.log; exit 1; }
}
ARGS="--camera C1"; run c1_def A=1; run c1_s4 VR_PATH=7 VR_SEG=4; run c1_s8 VR_PATH=7 VR_SEG=8
ARGS="--camera C0 --method 3"; run c0m3_def A=1; run c0m3_s4 VR_PATH=7 VR_SEG=4
ARGS="--camera C0 --method 2"; run c0m2_def A=1; run c0m2_s4 VR_PATH=7 VR_SEG=4
for f in $O/*.log; do echo "== $f"; grep -v amdgpu.ids $f | grep -v "tiles alone"; done
