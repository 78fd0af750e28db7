#!/bin/bash
# PMC passes of the baked march (C0, C1) and the headline march: issue, wait,
# TA/TD and cache counters, one rocprofv3 process per counter set.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/pmcb; mkdir -p $O
i=0
while read -r CTRS; do
  i=$((i+1))
  for W in "C0 --baked" "C1 --baked" "C0"; do
    N=$(echo $W | tr -d ' -')
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/$N/p$i -o p$i -- python bench.py --camera $W --no-cpu-baseline --no-issue-bounds --steps 3 --warmup 1 > $O/${N}_p$i.log 2>&1 || { echo "pass $i $N failed"; tail -5 $O/${N}_p$i.log; exit 1; }
  done
done < tools/pmc_sets.txt
echo done
