#!/bin/bash
# PMC passes over the GMM march (512^3 x K16, C0, method 1).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/gmmpmc; mkdir -p $O
CMD="python tools/gmm_time.py --dim 512 --cams C0 --methods 1 --reps 3"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- $CMD > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d $O/p1 -o p1 -- $CMD > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p2 -o p2 -- $CMD > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $O/p3 -o p3 -- $CMD > $O/p3.log 2>&1 || { tail $O/p3.log; exit 1; }
python3 tools/pmc_summary.py $O k_march_gmm
find $O/kt -name "*kernel_stats.csv" -exec grep -h "k_march_gmm" {} +
