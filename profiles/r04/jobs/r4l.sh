#!/bin/bash
# round 4, job l: K samples per footprint box (k_march_duo<B,M,K>) -- parity, then timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "duo or every_kernel_path" > $O/pytest_r4l.log 2>&1 || { tail -30 $O/pytest_r4l.log; exit 1; }
tail -1 $O/pytest_r4l.log
for M in 1 2; do
  timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method $M --rounds 5 --env "VR_DUO=0" "" "VR_DUO=3" "VR_DUO=4" > $O/variants_512x8_m$M.log 2>&1 || exit 1
  grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
done
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0 --method 1 --variants main --rounds 3 --env "" "VR_PATH=1,VR_DUO=0" "VR_PATH=1" "VR_PATH=1,VR_DUO=3" > $O/variants_1024x8_m1.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_1024x8_m1.log
echo done
