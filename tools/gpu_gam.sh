#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gam && export TMPDIR=/tmp
O=gpurun_out/gam
timeout -k 10 400 python -u tools/bench_variants.py --cameras C0 --rounds 6 --method 1 > $O/ab_m1.log 2>&1 || { tail -30 $O/ab_m1.log; exit 1; }; grep -v amdgpu.ids $O/ab_m1.log | tail -5
