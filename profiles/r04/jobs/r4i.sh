#!/bin/bash
# round 4, job i: LDS-tiled axis copy and line-whole brick copy (tests + first-frame
# kernel times); config 3 occupancy variants of the LDS-box march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py > $O/pytest_r4i.log 2>&1 || { tail -30 $O/pytest_r4i.log; exit 1; }
tail -1 $O/pytest_r4i.log
for CAM in S C1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o $CAM -- python bench.py --camera $CAM --no-cpu-baseline --no-issue-bounds --steps 5 --warmup 2 > $O/bench_$CAM.log 2>&1 || { tail -20 $O/bench_$CAM.log; exit 1; }
  grep -h "axis_copy\|brick8" $O/ktrace/${CAM}_kernel_stats.csv
done
timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 1 --rounds 5 > $O/variants_512x8_m1.log 2>&1 || exit 1
cat $O/variants_512x8_m1.log
echo done
