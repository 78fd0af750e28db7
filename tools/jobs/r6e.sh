# round 6 final build: PMC passes + bench lines + rocprofv3 kernel traces (tools/gpu_round.sh)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
RANKSIM=0 bash tools/gpu_round.sh ${1:-r6e} ${@:2}
