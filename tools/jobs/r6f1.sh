# round 6 session 3: whole GPU suite + smoke on the HEAD build, then the headline and baked workloads' PMC passes, bench lines and kernel traces
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_suite.sh r6f1 || exit 1
RANKSIM=0 bash tools/gpu_round.sh r6f1 1024x8:C0 1024x8:C0:baked 1024x8:C1:baked 128x1:C0 || exit 1
echo ok
