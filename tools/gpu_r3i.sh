#!/bin/bash
# Round-3: parity after the box-map default and the 32-bin box rule; config-3 and 32-bin bench lines.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3i}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_baked.py -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
tail -1 $O/pytest.log
for A in "--config 512x8" "--config 512x8 --method 2" "--config 1024x32 --no-cpu-baseline" "--config 1024x32 --method 3 --no-cpu-baseline --steps 5"; do
  timeout -k 10 400 python -u bench.py $A > $O/bench.log 2>&1; guard $? bench $O/bench.log
  echo "$A: $(grep -o '"ms_per_step": [0-9.]*\|"kernel": "[^"]*", "kernel_ms": [0-9.]*\|"rgba8_mismatch": [0-9]*' $O/bench.log | tr '\n' ' ')"
done
echo done
