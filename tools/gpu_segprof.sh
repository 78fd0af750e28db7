#!/bin/bash
# PMC passes 1-3 of tools/pmc_sets.txt for the default march and seg variants (full frame, C0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_def.log 2>&1 || exit 1
tail -1 gpurun_out/bench_def.log
BENCH="bench.py --config 1024x8 --steps 2 --warmup 1 --no-cpu-baseline"
for V in def 4 -4 -2; do
  if [ $V = def ]; then unset VR_PATH VR_SEG; else export VR_PATH=7 VR_SEG=$V; fi
  i=0
  head -3 tools/pmc_sets.txt | while read -r CTRS; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/seg$V/p$i -o s -- python $BENCH > gpurun_out/pmc/seg$V.p$i.log 2>&1 || { echo "fail $V $i"; exit 1; }
  done || exit 1
done
for V in def 4 -4 -2; do echo "== $V"; python tools/pmc_summary.py gpurun_out/pmc/seg$V k_march; done
