cd $GRAFT_REPO_ROOT
bash tools/gpu_pmc_bin.sh replay tools/build/replay_loads || exit $?
bash tools/gpu_pmc_bin.sh gbw tools/build/gather_bw || exit $?
