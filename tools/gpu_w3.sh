#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/w3 && export TMPDIR=/tmp
O=gpurun_out/w3
for m in 1 2; do timeout -k 10 300 python -u tools/bench_variants.py --cameras C0 --rounds 5 --method $m > $O/ab_m$m.log 2>&1 || { tail -30 $O/ab_m$m.log; exit 1; }; grep -v amdgpu.ids $O/ab_m$m.log | tail -3; done
