# round 6: the GPU suite + smoke on the pruned / split library, then the headline bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
bash tools/gpu_suite.sh r6b || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_n1.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config 512x8 --no-cpu-baseline > $O/bench_512.log 2>&1 || exit 1
echo ok
