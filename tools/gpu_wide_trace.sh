#!/bin/bash
# rocprofv3 kernel-trace stats of the wide-record bench commands (32 bins C0 / C1, 16 bins C0)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wtrace && export TMPDIR=/tmp
for A in "1024x32 C0" "1024x32 C1" "1024x16 C0"; do
  set -- $A
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wtrace -o $1_$2 -- python bench.py --config $1 --camera $2 --no-cpu-baseline --steps 10 > gpurun_out/wtrace/$1_$2.log 2>&1 || { tail -5 gpurun_out/wtrace/$1_$2.log; exit 1; }
  tail -1 gpurun_out/wtrace/$1_$2.log | cut -c1-200
done
