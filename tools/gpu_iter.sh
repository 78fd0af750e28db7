#!/bin/bash
# Iteration pass: GPU parity tests, then bench variants (C0/C1, staged box on/off).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
guard() { rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; guard $rc
[ $rc -ne 0 ] && exit $rc
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for cam in C0 C1; do
  for box in 1024 0; do
    VR_BOX_MAX=$box timeout -k 10 300 $B --camera $cam > gpurun_out/bench_${cam}_box${box}.log 2>&1; rc=$?; echo "bench $cam box=$box rc=$rc"; guard $rc
  done
done
echo done
