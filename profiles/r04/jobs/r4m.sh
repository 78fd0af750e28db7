#!/bin/bash
# round 4, job m: GPU suite after k_march_duo became the coarse-rows default; config 3 timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_r4m.log 2>&1 || { tail -30 $O/pytest_r4m.log; exit 1; }
tail -1 $O/pytest_r4m.log
timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 5 --env "VR_DUO=0" "" > $O/variants_512x8_m1.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_512x8_m1.log
echo done
