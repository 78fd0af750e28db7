cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_variants.py --rounds 3 --cameras C0 --env "" > gpurun_out/sweep.log 2> gpurun_out/sweep.err || exit $?
timeout -k 10 600 python -u tools/rank_sim.py --camera C0 > gpurun_out/ranks.log 2>&1 || exit $?
VRDD_LIB=tools/build/variants/nopf/libvr.so timeout -k 10 600 python -u tools/rank_sim.py --camera C0 >> gpurun_out/ranks.log 2>&1 || exit $?
