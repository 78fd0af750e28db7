#!/bin/bash
# round 4 final build: bench lines + kernel traces + PMC passes for the workloads given
# (split over several calls: gpurun's per-call limit).  usage: bash tools/jobs/r4_final_pmc.sh TAG workload...
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=$1; shift
RANKSIM=0 bash tools/gpu_round.sh $TAG "$@"
