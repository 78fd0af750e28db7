#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
RANKSIM=0 bash tools/gpu_round.sh r07b 1024x8:C0:baked 1024x8:C1:baked 256x4:C0 256x4:C0::2 128x1:C0 gmm1024:C0 1024x8:C0::3 1024x8:C1::3 256x4:C0::3 128x1:C0::3
