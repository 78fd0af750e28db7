#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
RANKSIM=0 bash tools/gpu_round.sh r07c 1024x32:C0::3 1024x32:C1::3 1024x16:C0::3 512x32:C0::3 512x8:C0::3
