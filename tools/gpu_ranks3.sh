cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -f gpurun_out/ranks.log
VR_PATH=1 VR_BOX_MAX=0 timeout -k 10 600 python -u tools/rank_sim.py --camera C0 >> gpurun_out/ranks.log 2>&1 || exit $?
VR_PATH=2 timeout -k 10 600 python -u tools/rank_sim.py --camera C0 >> gpurun_out/ranks.log 2>&1 || exit $?
