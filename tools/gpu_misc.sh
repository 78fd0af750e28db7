#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 tools/build/gather_bw > gpurun_out/gather_bw.log 2>&1 || exit $?
cp tools/pmc_sets.txt /tmp/pmc_all.txt
printf "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum\nTCC_EA0_RDREQ_128B_sum TCC_REQ_sum TCC_READ_sum TCC_HIT_sum\n" > tools/pmc_sets.txt
VR_BOX_MAX=1024 bash tools/gpu_prof.sh dram; rc=$?
cp /tmp/pmc_all.txt tools/pmc_sets.txt
exit $rc
