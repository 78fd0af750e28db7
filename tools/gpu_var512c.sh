#!/bin/bash
# Path sweep for coarse row-aligned views (LDS-box k_march vs the pipelined march)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/var512c; mkdir -p $O
for C in 128x1 256x4; do for M in 1 2; do
timeout -k 10 300 python -u tools/bench_variants.py --config $C --rounds 3 --method $M --cameras C0,C1 --env "" "VR_PATH=1" > $O/var_${C}_m$M.log 2>&1 || { tail -20 $O/var_${C}_m$M.log; exit 1; }
grep -v "round\|amdgpu" $O/var_${C}_m$M.log
done; done
