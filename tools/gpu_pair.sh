cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf -k "every_kernel_path" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/bench_variants.py --rounds 3 --cameras C0 --env VR_PATH=2 VR_PATH=6 > gpurun_out/sweep.log 2> gpurun_out/sweep.err || exit $?
VR_PATH=6 timeout -k 10 600 python -u tools/rank_sim.py --camera C0 > gpurun_out/ranks.log 2>&1 || exit $?
