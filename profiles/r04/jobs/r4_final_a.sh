#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
RANKSIM=0 bash tools/gpu_round.sh r07a 1024x8:C0 1024x8:C1 1024x8:S 1024x8:S:baked 512x8:C0 512x8:C0::2
