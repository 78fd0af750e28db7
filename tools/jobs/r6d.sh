# round 6: baked-plane copies kept per (axis, method); 36-byte GMM alive-list entries
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_baked.py tests/test_gpu_layout.py tests/test_gpu_gmm.py tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --config gmm2048 --slab-rehearsal --segments 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/rehearsal.log 2>&1; rc=$?; tail -c 600 $O/rehearsal.log; exit $rc
