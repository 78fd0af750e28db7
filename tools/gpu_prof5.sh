#!/bin/bash
cd $GRAFT_REPO_ROOT
VR_PATH=4 bash tools/gpu_prof.sh wsC0 --camera C0 || exit $?
VR_PATH=3 bash tools/gpu_prof.sh wgC0 --camera C0 || exit $?
VR_PATH=2 bash tools/gpu_prof.sh pipe16C0 --camera C0 || exit $?
