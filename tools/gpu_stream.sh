#!/bin/bash
# Out-of-core GMM streaming: parity + timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/stream; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gmm.py -k "stream" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for M in 1 2; do
timeout -k 10 400 python -u tools/gmm_stream_bench.py --dim 512 --slab 64 --method $M --check --incore > $O/m$M.log 2>&1 || { tail -20 $O/m$M.log; exit 1; }
grep "^{" $O/m$M.log
done
timeout -k 10 500 python -u tools/gmm_stream_bench.py --dim 768 --slab 64 --method 1 --frames 2 --incore > $O/d768.log 2>&1 || { tail -20 $O/d768.log; exit 1; }
grep "^{" $O/d768.log
