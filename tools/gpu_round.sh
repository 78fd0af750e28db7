#!/bin/bash
# Round measurement: GPU parity tests, bench lines (C0 default + C1), rocprofv3
# kernel-trace stats of the bench command, PMC traffic passes -> profiles/traffic.json.
# usage: bash tools/gpu_round.sh TAG [skip-tests]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; exit $rc; fi; }
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
timeout -k 10 600 python -u bench.py > $O/bench_1024x8_C0.log 2>&1; guard $? bench-C0
timeout -k 10 300 python -u bench.py --camera C1 --no-cpu-baseline > $O/bench_1024x8_C1.log 2>&1; guard $? bench-C1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o C0 -- python bench.py --no-cpu-baseline > $O/ktrace_C0.log 2>&1; guard $? ktrace-C0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o C1 -- python bench.py --camera C1 --no-cpu-baseline > $O/ktrace_C1.log 2>&1; guard $? ktrace-C1
for CAM in C0 C1; do
  i=0
  for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_$CAM/p$i -o p$i -- python bench.py --camera $CAM --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_${CAM}_p$i.log 2>&1; guard $? pmc-$CAM-$i
  done
  python tools/pmc_traffic.py $O/traffic.json "1024x8|$CAM|m1" $O/pmc_${CAM}_p1.log $O/pmc_$CAM/p1 $O/pmc_$CAM/p2 $O/pmc_$CAM/p3 || exit 1
done
# baked statistics (basicDataProcessing): bench, kernel trace, traffic
timeout -k 10 300 python -u bench.py --baked --no-cpu-baseline > $O/bench_1024x8_C0_baked.log 2>&1; guard $? bench-baked
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o C0_baked -- python bench.py --baked --no-cpu-baseline > $O/ktrace_C0_baked.log 2>&1; guard $? ktrace-baked
i=0
for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_C0_baked/p$i -o p$i -- python bench.py --baked --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_C0_baked_p$i.log 2>&1; guard $? pmc-baked-$i
done
python tools/pmc_traffic.py $O/traffic.json "1024x8|C0|m1|baked" $O/pmc_C0_baked_p1.log $O/pmc_C0_baked/p1 $O/pmc_C0_baked/p2 $O/pmc_C0_baked/p3 || exit 1
timeout -k 10 300 python -u bench.py --baked --camera C1 --no-cpu-baseline > $O/bench_1024x8_C1_baked.log 2>&1; guard $? bench-baked-C1
i=0
for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_C1_baked/p$i -o p$i -- python bench.py --baked --camera C1 --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_C1_baked_p$i.log 2>&1; guard $? pmc-baked-C1-$i
done
python tools/pmc_traffic.py $O/traffic.json "1024x8|C1|m1|baked" $O/pmc_C1_baked_p1.log $O/pmc_C1_baked/p1 $O/pmc_C1_baked/p2 $O/pmc_C1_baked/p3 || exit 1
for CAM in C0 C1; do
  timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM > $O/rank_sim_$CAM.log 2>&1; guard $? rank-sim-$CAM
done
echo done
