#!/bin/bash
# round 4, job ai: full-size rehearsal of the N = 2 bench loop (two render streams) on one
# GPU, tile gather staged through gloo: the assembled frame equals the single-rank frame
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4ai; mkdir -p $O
timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 --dump-frame $O/f1.npy > $O/bench_n1.log 2>&1 || { tail -20 $O/bench_n1.log; exit 1; }
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --no-cpu-baseline --steps 5 --warmup 2 --dist-backend gloo --dump-frame $O/f2.npy > $O/bench_n2_gloo.log 2>&1 || { tail -30 $O/bench_n2_gloo.log; exit 1; }
python -c "
import numpy as np; a=np.load('$O/f1.npy'); b=np.load('$O/f2.npy'); print('frames', a.shape, 'identical' if np.array_equal(a,b) else 'DIFFER %d' % int((a!=b).sum()))
" | tee $O/compare.log
grep '^{' $O/bench_n2_gloo.log | cut -c1-400
echo done
