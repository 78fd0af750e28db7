#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/var512b; mkdir -p $O
timeout -k 10 500 python -u tools/bench_variants.py --config 512x8 --rounds 3 --method 1 --cameras C0 --env "" "VR_PATH=6" "VR_PATH=5" "VR_PATH=1" "VR_PATH=3" "VR_WG_PER_CU=4" "VR_WG_PER_CU=2" > $O/var.log 2>&1 || { tail -20 $O/var.log; exit 1; }
grep -v "round\|amdgpu" $O/var.log
