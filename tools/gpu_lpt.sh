cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_variants.py --rounds 3 --env "" VR_NO_LPT=1 > gpurun_out/sweep.log 2> gpurun_out/sweep.err || exit $?
timeout -k 10 600 python -u tools/rank_sim.py --camera C0 > gpurun_out/ranks.log 2>&1 || exit $?
VR_NO_LPT=1 timeout -k 10 600 python -u tools/rank_sim.py --camera C0 --no-lpt >> gpurun_out/ranks.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/rank_sim.py --camera C1 >> gpurun_out/ranks.log 2>&1 || exit $?
