cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 tools/build/ea_calib > gpurun_out/ea_calib.log 2>&1 || exit $?
SETS=tools/pmc_sets_ea.txt bash tools/gpu_pmc_bin.sh ea tools/build/ea_calib || exit $?
