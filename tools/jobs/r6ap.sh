# round 6 final build: the whole GPU suite + smoke, the driver's default bench
# line (traffic from the committed profiles/traffic.json), and the N = 2 line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ap; mkdir -p $O
bash tools/gpu_suite.sh r6ap || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --gpus 2 --dist-backend gloo > $O/bench_n2_1024.log 2>&1 || exit 1
echo ok
