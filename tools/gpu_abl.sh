#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_variants.py --cameras C0 --rounds 6 > gpurun_out/abl/abl.log 2>&1 || { tail -30 gpurun_out/abl/abl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/abl/abl.log | tail -8
