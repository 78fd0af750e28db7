#!/bin/bash
# Baked method 7: kernel x occupancy cap
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked5; mkdir -p $O
timeout -k 10 400 python -u tools/bench_variants.py --baked --config 1024x8 --rounds 3 --method 7 --cameras C0,C1 --env "VR_M7_PIPE=0" "VR_M7_PIPE=0,VR_WG_PER_CU=2" "VR_M7_PIPE=0,VR_WG_PER_CU=3" "VR_M7_PIPE=0,VR_WG_PER_CU=4" "VR_M7_PIPE=0,VR_WG_PER_CU=6" "VR_WG_PER_CU=2" "VR_WG_PER_CU=1" > $O/m7_baked.log 2>&1 || { tail -20 $O/m7_baked.log; exit 1; }
grep -v "round\|amdgpu" $O/m7_baked.log
timeout -k 10 400 python -u tools/bench_variants.py --baked --config 512x8 --rounds 3 --method 7 --cameras C0,C1 --env "" "VR_M7_PIPE=0" "VR_M7_PIPE=0,VR_WG_PER_CU=2" "VR_WG_PER_CU=2" > $O/m7_baked512.log 2>&1 || { tail -20 $O/m7_baked512.log; exit 1; }
grep -v "round\|amdgpu" $O/m7_baked512.log
