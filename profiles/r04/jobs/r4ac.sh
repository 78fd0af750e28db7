#!/bin/bash
# round 4, job ac: configs 1 and 2 on the LDS-box march (one / two samples per box)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4ac; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1 --method 1 --rounds 5 --env "" "VR_PATH=1,VR_DUO=0" "VR_PATH=1,VR_DUO=2" "VR_PATH=1,VR_DUO=3" > $O/variants_256x4_box.log 2>&1 || { tail -20 $O/variants_256x4_box.log; exit 1; }
grep -v "round\|amdgpu.ids" $O/variants_256x4_box.log
timeout -k 10 600 python -u tools/bench_variants.py --config 128x1 --cameras C0,C1 --method 1 --rounds 5 --env "" "VR_PATH=1,VR_DUO=0" "VR_PATH=1,VR_DUO=2" > $O/variants_128x1_box.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_128x1_box.log
echo done
