#!/bin/bash
# PMC passes (tools/pmc_sets.txt) over a short 1024^3x8 bench; env knobs pass through.
# usage: tools/gpu_prof.sh TAG [extra bench args]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
TAG=${1:-r01}; shift
guard() { rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
BENCH="bench.py --config 1024x8 --steps 2 --warmup 1 --no-cpu-baseline $*"
i=0
while read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/$TAG/p$i -o $TAG -- python $BENCH > gpurun_out/pmc/$TAG.p$i.log 2>&1; rc=$?; echo "$TAG pass $i rc=$rc"; guard $rc
done < tools/pmc_sets.txt
