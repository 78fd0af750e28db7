#!/bin/bash
# round 4, job q: the final build's measurement, part 3 (wide records, entropy)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
RANKSIM=0 bash tools/gpu_round.sh r05c 1024x32:C0::3 1024x32:C1::3 1024x16:C0::3 512x32:C0::3 512x8:C0::3
