#!/bin/bash
# Bench lines for every BASELINE config that fits one GPU (configs 1-4; config 5 via gmm_slab_sim).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/configs; mkdir -p $O
for C in 128x1 256x4 512x8 1024x8; do
  timeout -k 10 300 python -u bench.py --config $C > $O/bench_$C.log 2>&1 || { tail $O/bench_$C.log; exit 1; }
  grep '^{' $O/bench_$C.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$C', d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
done
