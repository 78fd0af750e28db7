#!/bin/bash
# round 4, job k: two samples per footprint box (k_march_duo) -- parity, then config 3 timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "duo or every_kernel_path" > $O/pytest_r4k.log 2>&1 || { tail -30 $O/pytest_r4k.log; exit 1; }
tail -1 $O/pytest_r4k.log
for M in 1 2 3; do
  timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method $M --rounds 5 --env "" "VR_DUO=1" > $O/variants_512x8_m$M.log 2>&1 || exit 1
  grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
done
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 1 --variants main,g2 --rounds 3 --env "VR_PATH=1" "VR_PATH=1,VR_DUO=1" > $O/variants_1024x8_m1.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_1024x8_m1.log
echo done
