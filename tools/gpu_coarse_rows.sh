#!/bin/bash
# Coarse row-aligned heuristic: parity + default-path timings (profiles/r02/paths_coarse_rows.log)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/coarse_rows; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "coarse" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for M in 1 2 3; do
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --rounds 3 --method $M --cameras C0,C1 --env "" "VR_PATH=2" > $O/var_m$M.log 2>&1 || { tail -20 $O/var_m$M.log; exit 1; }
grep -v "round\|amdgpu" $O/var_m$M.log
done
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --rounds 3 --method 1 --cameras C0 --env "" > $O/var1024.log 2>&1 || { tail -20 $O/var1024.log; exit 1; }
grep -v "round\|amdgpu" $O/var1024.log
