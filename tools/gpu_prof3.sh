#!/bin/bash
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh quadC0 --camera C0 || exit $?
bash tools/gpu_prof.sh quadC1 --camera C1 || exit $?
VR_PATH=2 bash tools/gpu_prof.sh pipeC0 --camera C0 || exit $?
