#!/bin/bash
# Round-3: LDS-box chunking check (parity + 512^3 bench), VALU counter calibration,
# samples-per-pixel dumps for tools/footprint_sim.c.  usage: bash tools/gpu_r3c.sh [TAG]
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3c}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -20 $3; exit $rc; fi; }
mkdir -p tools/build && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/valu_calib.hip -o tools/build/valu_calib 2> /dev/null || exit 1
timeout -k 10 120 tools/build/valu_calib > $O/valu_calib.log 2>&1; guard $? calib $O/valu_calib.log
cat $O/valu_calib.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_calib -o calib -- tools/build/valu_calib > $O/pmc_calib.log 2>&1; guard $? pmc-calib $O/pmc_calib.log
timeout -k 10 300 python -u tools/dump_steps.py > $O/dump_steps.log 2>&1; guard $? dump $O/dump_steps.log
ls -la gpurun_out/steps_*.npy
echo done
