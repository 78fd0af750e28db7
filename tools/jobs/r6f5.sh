# round 6 session 3: the whole -m gpu suite and smoke() as the driver runs them (config-5 whole-frame default), then the driver-form bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_suite.sh r6f5 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r6f5/bench_default.log 2>&1 || exit 1
echo ok
