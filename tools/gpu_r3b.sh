#!/bin/bash
# Round-3 measurements (one gpurun call): rotation sweep of the kernel choice,
# bench lines + rocprofv3 kernel stats + PMC passes (traffic, issue) of the
# smaller BASELINE configs, the GMM march (config 5's kernel at 1024^3), and
# the multi-GPU rank simulation at steady state.  usage: bash tools/gpu_r3b.sh [TAG]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3b}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -20 $3; exit $rc; fi; }
timeout -k 10 300 python -u tools/rot_sweep.py > $O/rot_sweep_1024x8.log 2>&1; guard $? rot $O/rot_sweep_1024x8.log
for CFG in 128x1 256x4 512x8; do
  timeout -k 10 300 python -u bench.py --config $CFG > $O/bench_$CFG.log 2>&1; guard $? bench-$CFG $O/bench_$CFG.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o $CFG -- python bench.py --config $CFG --no-cpu-baseline > $O/ktrace_$CFG.log 2>&1; guard $? ktrace-$CFG $O/ktrace_$CFG.log
  i=0
  for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_$CFG/p$i -o p$i -- python bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_${CFG}_p$i.log 2>&1; guard $? pmc-$CFG-$i $O/pmc_${CFG}_p$i.log
  done
  PMC_TAG=r3b python tools/pmc_traffic.py $O/traffic.json "$CFG|C0|m1" $O/pmc_${CFG}_p1.log $O/pmc_$CFG/p1 $O/pmc_$CFG/p2 $O/pmc_$CFG/p3 > /dev/null || exit 1
done
timeout -k 10 400 python -u bench.py --config gmm1024 > $O/bench_gmm1024.log 2>&1; guard $? bench-gmm $O/bench_gmm1024.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o gmm1024 -- python bench.py --config gmm1024 --no-cpu-baseline > $O/ktrace_gmm1024.log 2>&1; guard $? ktrace-gmm $O/ktrace_gmm1024.log
i=0
for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_gmm1024/p$i -o p$i -- python bench.py --config gmm1024 --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_gmm1024_p$i.log 2>&1; guard $? pmc-gmm-$i $O/pmc_gmm1024_p$i.log
done
PMC_TAG=r3b python tools/pmc_traffic.py $O/traffic.json "gmm1024|C0|m1" $O/pmc_gmm1024_p1.log $O/pmc_gmm1024/p1 $O/pmc_gmm1024/p2 $O/pmc_gmm1024/p3 > /dev/null || exit 1
for CAM in C0 C1; do
  timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM > $O/rank_sim_$CAM.log 2>&1; guard $? rank-$CAM $O/rank_sim_$CAM.log
done
echo done
