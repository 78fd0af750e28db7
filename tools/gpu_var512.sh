#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/var512; mkdir -p $O
for M in 1 2 3; do
timeout -k 10 500 python -u tools/bench_variants.py --config 512x8 --rounds 3 --method $M --cameras C0,C1 --env "" "VR_PATH=2" "VR_PATH=4" "VR_PATH=0" "VR_PATH=7,VR_SEG=-2" "VR_PATH=7,VR_SEG=-4" > $O/var_m$M.log 2>&1 || { tail -20 $O/var_m$M.log; exit 1; }
grep -v "round\|amdgpu" $O/var_m$M.log
done
