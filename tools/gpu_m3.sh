cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_variants.py --rounds 2 --method 3 --env VR_PATH=1 VR_PATH=3 VR_PATH=4 > gpurun_out/m3.log 2> gpurun_out/m3.err || exit $?
timeout -k 10 600 python -u tools/bench_variants.py --rounds 2 --method 2 --env VR_PATH=1 VR_PATH=3 VR_PATH=4 >> gpurun_out/m3.log 2>> gpurun_out/m3.err || exit $?
