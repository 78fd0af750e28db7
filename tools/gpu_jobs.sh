#!/bin/bash
# Named GPU experiments of round 3 (each writes gpurun_out/<job>/ and is the
# source of the profiles/r03 log named beside it).  The round's bench lines,
# kernel traces and PMC passes: tools/gpu_round.sh; the GPU suite: tools/gpu_suite.sh.
#   bash tools/gpu_jobs.sh sweep   -> rot_sweep_1024x8*.log, rot_sweep_512x8_axis_copies.log
#   bash tools/gpu_jobs.sh calib   -> valu_calib.log, valu_calib_pmc.csv
#   bash tools/gpu_jobs.sh steps   -> gpurun_out/steps_C*.npy for tools/footprint_sim.c (footprint_planes.log)
#   bash tools/gpu_jobs.sh box     -> box_map.log (LDS-box march: wave maps, wide records, oblique views)
#   bash tools/gpu_jobs.sh ranks   -> rank_sim_1024x8_C*.log
#   bash tools/gpu_jobs.sh quad2   -> quad2 parity, C1 rank wave timelines, rank_sim_1024x8_C1_quad2.log
#   bash tools/gpu_jobs.sh segc0   -> C0 rank lists: wave timeline and the ray-segmented variants
#   bash tools/gpu_jobs.sh baked   -> baked full frames: wave timeline, segmented / pipelined variants
#   bash tools/gpu_jobs.sh pmcb    -> pmc_issue_baked_vs_headline.log (tools/pmc_sets.txt passes; summary:
#                                     tools/pmc_summary.py gpurun_out/pmcb/<C0baked|C1baked|C0> <kernel>)
#   bash tools/gpu_jobs.sh wide    -> bench_1024x16_*, bench_1024x32_*, bench_512x32_* (no CPU baseline)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
J=${1:?job}; O=gpurun_out/$J; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
case $J in
sweep)
  timeout -k 10 400 python -u tools/rot_sweep.py --rx 0,30,90 --step 10 > $O/rot_1024x8.log 2>&1; guard $? rot $O/rot_1024x8.log
  timeout -k 10 300 python -u tools/rot_sweep.py --config 512x8 --rx 0 --step 10 --paths 7 > $O/rot_512x8.log 2>&1; guard $? rot512 $O/rot_512x8.log ;;
calib)
  mkdir -p tools/build && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/valu_calib.hip -o tools/build/valu_calib 2> /dev/null || exit 1
  timeout -k 10 120 tools/build/valu_calib > $O/valu_calib.log 2>&1; guard $? calib $O/valu_calib.log
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o calib -- tools/build/valu_calib > $O/pmc.log 2>&1; guard $? pmc $O/pmc.log ;;
steps)
  timeout -k 10 300 python -u tools/dump_steps.py > $O/dump.log 2>&1; guard $? dump $O/dump.log ;;
box)
  for CC in 512x8:1:C0 512x8:2:C0 1024x8:1:C0 1024x16:1:C0 1024x16:2:C0 1024x16:3:C0 1024x32:1:C0 1024x32:2:C0 1024x32:3:C0 512x8:1:C1 1024x32:1:C1; do
    IFS=: read CFG M CAM <<< "$CC"
    timeout -k 10 400 python -u tools/bench_variants.py --config $CFG --rounds 2 --reps 3 --method $M --cameras $CAM --env "" "VR_PATH=1" "VR_PATH=1,VR_BOX_MAP=0" > $O/box_${CFG}_m${M}_$CAM.log 2>&1; guard $? box-$CC $O/box_${CFG}_m${M}_$CAM.log
  done ;;
ranks)
  for CAM in C0 C1; do
    timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM > $O/rank_sim_$CAM.log 2>&1; guard $? rank-$CAM $O/rank_sim_$CAM.log
  done ;;
quad2)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "quad_two_lanes or (every_kernel_path and QUAD2)" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  for E in "" VR_QUAD2=1; do
    timeout -k 10 300 python -u tools/wave_timeline.py --camera C1 --world 8 --ranks 0,3 --env "$E" --cost > $O/wt_$E.log 2>&1; guard $? wt $O/wt_$E.log
  done
  for E in "" VR_QUAD2=1 VR_QUAD2=1,VR_WG_PER_CU=2 VR_QUAD2=1,VR_WG_PER_CU=3; do
    timeout -k 10 300 python -u tools/rank_sim.py --camera C1 --env "$E" > $O/rs_$E.log 2>&1; guard $? rs $O/rs_$E.log
  done ;;
segc0)
  timeout -k 10 300 python -u tools/wave_timeline.py --camera C0 --world 8 --ranks 0,3 --env "" --cost > $O/wt.log 2>&1; guard $? wt $O/wt.log
  for E in "" VR_SEG=-4 VR_SEG=4 VR_WG_PER_CU=3 VR_WG_PER_CU=4 VR_SEG=-4,VR_WG_PER_CU=4; do
    timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --env "$E" > $O/rs_$E.log 2>&1; guard $? rs $O/rs_$E.log
  done ;;
baked)
  timeout -k 10 300 python -u tools/wave_timeline.py --camera C0 --world 8 --ranks 0 --env "" --cost --baked > $O/wt.log 2>&1; guard $? wt $O/wt.log
  timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --baked --rounds 3 --reps 5 --cameras C0,C1 --env "" VR_PATH=2 VR_PATH=7,VR_SEG=-2 VR_PATH=7,VR_SEG=2 VR_PATH=7,VR_SEG=4 VR_PATH=7,VR_SEG=-4 > $O/variants.log 2>&1; guard $? var $O/variants.log ;;
pmcb)
  i=0
  while read -r CTRS; do
    i=$((i+1))
    for W in "C0 --baked" "C1 --baked" "C0"; do
      N=$(echo $W | tr -d ' -')
      timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O/$N/p$i -o p$i -- python bench.py --camera $W --no-cpu-baseline --no-issue-bounds --steps 3 --warmup 1 > $O/${N}_p$i.log 2>&1; guard $? pmc-$N-$i $O/${N}_p$i.log
    done
  done < tools/pmc_sets.txt ;;
wide)
  for W in "1024x32 C0 1" "1024x32 C1 1" "1024x32 C0 3" "1024x16 C0 1" "1024x16 C1 1" "512x32 C0 1" "512x32 C1 1"; do
    read CFG CAM M <<< "$W"
    timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method $M --no-cpu-baseline > $O/bench_${CFG}_${CAM}_m$M.log 2>&1; guard $? wide-$CFG $O/bench_${CFG}_${CAM}_m$M.log
  done ;;
*) echo "unknown job $J"; exit 2 ;;
esac
echo done
