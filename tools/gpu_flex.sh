#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/flex && export TMPDIR=/tmp
O=gpurun_out/flex
timeout -k 10 300 python -u tools/flex_time.py > $O/flex_time.log 2>&1 || { cat $O/flex_time.log; exit 1; }
grep -v amdgpu.ids $O/flex_time.log
