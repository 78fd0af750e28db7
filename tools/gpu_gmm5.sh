#!/bin/bash
# GMM: bench N=2 (gloo, balanced re-cut) vs N=1, then config-5 slab simulation with the cost re-cut.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/gmm5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
timeout -k 10 900 python -u tools/gmm_slab_sim.py --balance > $O/sim2048_bal.log 2>&1 || { cat $O/sim2048_bal.log; exit 1; }
grep -v amdgpu.ids $O/sim2048_bal.log
