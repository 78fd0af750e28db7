#!/bin/bash
# Quad codec march: parity (codec tests on oblique views) + C1 timings quad vs one-lane.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/cquad; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k codec -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit 1; }
for M in 4 5 6; do for Q in 0 1; do
  VR_CODEC_QUAD=$Q timeout -k 10 240 python -u bench.py --method $M --camera C1 --no-cpu-baseline > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  echo "C1 m$M quad=$Q: $(grep -o '"kernel_ms": [0-9.]*' $O/b.log) $(grep -o '"value": [0-9.]*' $O/b.log | head -1) $(grep -o '"kernel": "[^"]*' $O/b.log)"
done; done
