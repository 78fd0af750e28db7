#!/bin/bash
cd $GRAFT_REPO_ROOT
VR_BOX_MAX=1024 bash tools/gpu_prof.sh staged || exit $?
VR_BOX_MAX=0 VR_WG_PER_CU=2 bash tools/gpu_prof.sh direct || exit $?
