#!/bin/bash
# round 4, job j: config 3 -- box chunk size and occupancy variants of the LDS-box march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
for M in 1 2 3; do
  timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method $M --rounds 5 > $O/variants_512x8_m$M.log 2>&1 || exit 1
  grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
done
echo done
