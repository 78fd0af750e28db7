#!/bin/bash
# baked C1: lanes per ray x occupancy cap (narrow pair gathers)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked7; mkdir -p $O
timeout -k 10 500 python -u tools/bench_variants.py --baked --config 1024x8 --rounds 3 --method 1 --cameras C1 --env "" "VR_WG_PER_CU=4" "VR_WG_PER_CU=5" "VR_WG_PER_CU=6" "VR_WG_PER_CU=8" "VR_SEG=2,VR_WG_PER_CU=4" "VR_SEG=8,VR_WG_PER_CU=6" > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
grep -v "round\|amdgpu" $O/c1.log
timeout -k 10 500 python -u tools/bench_variants.py --baked --config 1024x8 --rounds 3 --method 1 --cameras C0 --env "" "VR_WG_PER_CU=5" "VR_WG_PER_CU=6" > $O/c0.log 2>&1 || { tail -20 $O/c0.log; exit 1; }
grep -v "round\|amdgpu" $O/c0.log
timeout -k 10 500 python -u tools/bench_variants.py --baked --config 512x8 --rounds 3 --method 1 --cameras C1 --env "" "VR_WG_PER_CU=8" "VR_WG_PER_CU=6" > $O/c1_512.log 2>&1 || { tail -20 $O/c1_512.log; exit 1; }
grep -v "round\|amdgpu" $O/c1_512.log
