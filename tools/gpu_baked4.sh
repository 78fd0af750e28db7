#!/bin/bash
# Baked method 7 + full GPU suite
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked4; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --rounds 3 --method 7 --cameras C0,C1 --env "" > $O/m7_records.log 2>&1 || { tail -20 $O/m7_records.log; exit 1; }
grep -v "round\|amdgpu" $O/m7_records.log
timeout -k 10 300 python -u tools/bench_variants.py --baked --config 1024x8 --rounds 3 --method 7 --cameras C0,C1 --env "" "VR_WG_PER_CU=2" "VR_WG_PER_CU=3" "VR_M7_PIPE=0" > $O/m7_baked.log 2>&1 || { tail -20 $O/m7_baked.log; exit 1; }
grep -v "round\|amdgpu" $O/m7_baked.log
