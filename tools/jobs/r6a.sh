cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gmm.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --gpus 2 --config 256x4 --dist-backend gloo > $O/bench_n2_256.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --gpus 2 --config 1024x8 --dist-backend gloo > $O/bench_n2_1024.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_n1.log 2>&1 || exit 1
echo ok
