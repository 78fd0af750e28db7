#!/bin/bash
# round 4, job ab: oblique wide-record entropy on the LDS-box march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4ab; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x32 --cameras C1 --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=1" > $O/variants_1024x32_C1_m3.log 2>&1 || { tail -20 $O/variants_1024x32_C1_m3.log; exit 1; }
grep -v "round\|amdgpu.ids" $O/variants_1024x32_C1_m3.log
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x16 --cameras C1 --method 3 --rounds 3 --reps 2 --env "" "VR_PATH=1" > $O/variants_1024x16_C1_m3.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_1024x16_C1_m3.log
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x32 --cameras C1 --method 1 --rounds 2 --reps 2 --env "" "VR_PATH=1" > $O/variants_1024x32_C1_m1.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_1024x32_C1_m1.log
echo done
