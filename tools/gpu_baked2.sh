#!/bin/bash
# Baked march look-ahead depth sweep (VR_BAKED_DEPTH) + parity
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_baked.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for C in 1024x8 512x8; do
timeout -k 10 400 python -u tools/bench_variants.py --baked --config $C --rounds 3 --method 1 --cameras C0,C1 --env "VR_BAKED_DEPTH=1" "VR_BAKED_DEPTH=2" "VR_BAKED_DEPTH=3" "" "VR_BAKED_DEPTH=6" "VR_BAKED_DEPTH=8" "VR_BAKED_DEPTH=4,VR_WG_PER_CU=4" "VR_PATH=7,VR_SEG=4" > $O/var_$C.log 2>&1 || { tail -20 $O/var_$C.log; exit 1; }
grep -v "round\|amdgpu" $O/var_$C.log
done
