#!/bin/bash
# round 4, job n: config 3 (k_march_duo) against the full-frame tile order (XCD blocks, LPT)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 5 --env "" "VR_NO_LPT=1" "VR_XBLOCK=0" "VR_XBLOCK=4,4" "VR_XBLOCK=8,8" "VR_XBLOCK=2,16" "VR_XBLOCK=4,4,VR_NO_LPT=1" "VR_XBLOCK=8,8,VR_NO_LPT=1" > $O/variants_512x8_order.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_512x8_order.log
echo done
