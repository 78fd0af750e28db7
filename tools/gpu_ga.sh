#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ga && export TMPDIR=/tmp
O=gpurun_out/ga
for m in 1 2; do timeout -k 10 400 python -u tools/bench_variants.py --cameras C0 --rounds 5 --method $m > $O/ab_m$m.log 2>&1 || { tail -30 $O/ab_m$m.log; exit 1; }; grep -v amdgpu.ids $O/ab_m$m.log | tail -5; done
