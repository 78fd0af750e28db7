#!/bin/bash
# GMM bench mode + slab simulation (check at 512^3, then config 5 at 2048^3).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/gmm4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
timeout -k 10 300 python -u tools/gmm_slab_sim.py --dim 512 --W 1920 --H 1080 --check > $O/sim512.log 2>&1 || { cat $O/sim512.log; exit 1; }
grep -v amdgpu.ids $O/sim512.log | tail -3
timeout -k 10 400 python -u bench.py --config gmm1024 > $O/bench_gmm1024.log 2>&1 || { tail -20 $O/bench_gmm1024.log; exit 1; }
tail -1 $O/bench_gmm1024.log
timeout -k 10 600 python -u tools/gmm_slab_sim.py > $O/sim2048.log 2>&1 || { cat $O/sim2048.log; exit 1; }
grep -v amdgpu.ids $O/sim2048.log
