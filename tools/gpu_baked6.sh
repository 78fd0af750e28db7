#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked6; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_baked.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/bench_variants.py --baked --config 512x8 --rounds 3 --method 7 --cameras C0,C1 --env "" "VR_WG_PER_CU=0" > $O/m7_512.log 2>&1 || { tail -20 $O/m7_512.log; exit 1; }
grep -v "round\|amdgpu" $O/m7_512.log
