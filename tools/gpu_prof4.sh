cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh q2C0 --camera C0 || exit $?
