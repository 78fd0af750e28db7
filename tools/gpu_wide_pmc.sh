#!/bin/bash
# PMC passes over the wide-record march (1024^3 x 32, C0, method 1): TA / TCP busy
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/widepmc && export TMPDIR=/tmp
i=0
for CTRS in "TA_TA_BUSY_sum TA_BUSY_max GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" \
            "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
            "TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/widepmc/p$i -o p$i -- python bench.py --config ${CFG:-1024x32} --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/widepmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/widepmc/p$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/widepmc ${KPAT:-k_march_w} 2>&1 | tail -30
