#!/bin/bash
# round 4, job e: wide entropy (rolled LDS columns in k_march / k_march_wq), box reciprocals, loop-overhead sources
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_random.py > $O/pytest_r4e.log 2>&1 || { tail -30 $O/pytest_r4e.log; exit 1; }
tail -2 $O/pytest_r4e.log
for A in "1024x32:C0:3" "1024x32:C1:3" "1024x16:C0:3" "1024x16:C1:3" "512x8:C0:1" "1024x32:C0:1"; do
  IFS=: read CFG CAM MTH <<< "$A"
  timeout -k 10 400 python -u bench.py --config $CFG --camera $CAM --method $MTH --no-cpu-baseline > $O/bench_${CFG}_${CAM}_m$MTH.log 2>&1 || exit 1
done
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=4" > $O/variants_1024x8_m3.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=4" > $O/variants_512x8_m3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8.log 2>&1 || exit 1
echo done
