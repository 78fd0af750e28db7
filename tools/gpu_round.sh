#!/bin/bash
# Round measurement: for every workload the PMC passes -- FETCH_SIZE, WRITE_SIZE,
# TCC_EA0 requests, VALU issue -- run one per process (MI355X_MICROARCH.md PMC
# slot limits) and folded into traffic.json (tools/pmc_traffic.py, keyed by
# workload and by the sha256 of this libvr.so), then the bench line (with the CPU
# baseline and parity check) reading that traffic.json, so the line carries its
# own build's traffic, then the rocprofv3 --kernel-trace --stats summary of the
# same bench command.  Then the steady-state rank simulation.
# usage: bash tools/gpu_round.sh TAG [workload ...]   (workload = config:camera[:baked[:method]],
#   e.g. 1024x32:C0::3 for method 3 per-step, 1024x8:S:baked)
#   PMC=0: bench lines and kernel traces only (profiles/traffic.json already holds
#   this build's passes); RANKSIM=0: no rank simulation.  Run the PMC passes of one
#   build in ONE call, or merge their traffic.json files: each call starts from a
#   fresh gpurun_out/ on the box.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${1:-r03}; shift
O=gpurun_out/$TAG; mkdir -p $O
WL=${@:-"1024x8:C0 1024x8:C1 1024x8:S 1024x8:C0:baked 1024x8:C1:baked 512x8:C0 256x4:C0 128x1:C0 gmm1024:C0"}
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -20 $3; exit $rc; fi; }
for W in $WL; do
  IFS=: read CFG CAM BK MTH <<< "$W"
  MTH=${MTH:-1}
  ARGS="--config $CFG --camera $CAM --method $MTH"; KEY="$CFG|$CAM|m$MTH"; N="${CFG}_$CAM"
  [ "$MTH" != 1 ] && N="${N}_m$MTH"
  if [ "$BK" = baked ]; then ARGS="$ARGS --baked"; KEY="$KEY|baked"; N="${N}_baked"; fi
  # PMC passes first, so the bench line of this same build carries their traffic
  if [ "${PMC:-1}" = 1 ]; then
  i=0
  for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_$N/p$i -o p$i -- python bench.py $ARGS --no-cpu-baseline --no-issue-bounds --steps 3 --warmup 1 > $O/pmc_${N}_p$i.log 2>&1; guard $? pmc-$N-$i $O/pmc_${N}_p$i.log
  done
  PMC_TAG=$TAG python tools/pmc_traffic.py $O/traffic.json "$KEY" $O/pmc_${N}_p1.log $O/pmc_$N/p1 $O/pmc_$N/p2 $O/pmc_$N/p3 $O/pmc_$N/p4 > /dev/null || exit 1
  TJ="--traffic-json $O/traffic.json"
  fi
  timeout -k 10 900 python -u bench.py $ARGS ${TJ:-} > $O/bench_$N.log 2>&1; guard $? bench-$N $O/bench_$N.log
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o $N -- python bench.py $ARGS --no-cpu-baseline --no-issue-bounds > $O/ktrace_$N.log 2>&1; guard $? ktrace-$N $O/ktrace_$N.log
  echo "$N $(grep -o '"kernel": "[^"]*", "kernel_ms": [0-9.]*' $O/bench_$N.log)"
done
if [ "${RANKSIM:-1}" = 1 ]; then
  for CAM in C0 C1 S; do
    timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM > $O/rank_sim_$CAM.log 2>&1; guard $? rank-sim-$CAM $O/rank_sim_$CAM.log
  done
fi
echo done
