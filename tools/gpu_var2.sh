#!/bin/bash
# A/B of tools/build/variants/* against the in-tree build (bench_variants.py).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/var2; mkdir -p $O
for M in ${METHODS:-1}; do
timeout -k 10 500 python -u tools/bench_variants.py --config 1024x8 --rounds 5 --method $M > $O/var_m$M.log 2>&1 || { tail -20 $O/var_m$M.log; exit 1; }
grep -v "round\|amdgpu" $O/var_m$M.log
done
