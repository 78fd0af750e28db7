#!/bin/bash
# Round-5 GPU jobs, one case per gpurun call: bash tools/jobs/r5.sh <job>
# (each writes gpurun_out/<job>/; the committed logs under profiles/r05/ name
# the job they came from).  Round 4's single-use scripts: profiles/r04/jobs/.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
J=${1:?job}; O=gpurun_out/$J; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
# a heartbeat file under gpurun_out: tests that run bench.py as a subprocess print
# nothing for minutes on a fresh box (first torch import); every step still has
# its own timeout, so a real hang ends there
( while sleep 50; do date >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -c "import torch; print('torch', torch.__version__, torch.cuda.is_available())" || exit 1
case $J in
launch)  # self-launched N = 2 bench, layout / wide-plane tests, m3 rank-list paths
  timeout -k 10 600 $PYT tests/test_gpu_bench.py tests/test_gpu_layout.py > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -3 $O/pytest.log
  timeout -k 10 300 python -u bench.py --gpus 2 --config 256x4 --dist-backend gloo --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_n2.log 2>&1; guard $? n2 $O/bench_n2.log
  grep '^{' $O/bench_n2.log | cut -c1-400
  for CAM in C0; do
    timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM --method 3 --modes cost --envs "" "VR_PATH=4" > $O/rank_m3_$CAM.log 2>&1; guard $? rs-m3 $O/rank_m3_$CAM.log
  done ;;
duo)  # k_march_duo entropy restored: parity, LDS-box bound check (checking build), timing
  [ -n "$SKIP_PYTEST" ] || { timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "duo or every_kernel_path" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log; }
  VRDD_LIB=tools/build/variants/boxcheck/libvr.so timeout -k 10 300 python -u tools/box_check.py > $O/box_check.log 2>&1; guard $? boxcheck $O/box_check.log
  tail -3 $O/box_check.log
  for CFG in 512x8 1024x8; do
    timeout -k 10 400 python -u tools/bench_variants.py --variants main --config $CFG --cameras C0 --method 3 --rounds 3 --env "" "VR_PATH=1,VR_DUO=2" "VR_PATH=1,VR_DUO=3" "VR_PATH=1,VR_DUO=4" > $O/variants_${CFG}_m3.log 2>&1; guard $? var $O/variants_${CFG}_m3.log
    grep -v "round\|amdgpu.ids" $O/variants_${CFG}_m3.log
  done ;;
gmm5)  # BASELINE config 5 rehearsed on one GPU: every slab of the 8-slab chain timed
  timeout -k 10 600 $PYT tests/test_gpu_gmm.py -k "not at_size" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  timeout -k 10 1000 python -u bench.py --config gmm2048 --slab-rehearsal --steps 5 --warmup 1 > $O/bench.log 2>&1; guard $? gmm5 $O/bench.log
  grep '^{' $O/bench.log | cut -c1-600 ;;
ranks)  # every rank's bench.py frame loop replayed: max over ranks, host + staged peer copies in
  for CAM in C0 C1; do for N in 2 4 8; do
    timeout -k 10 300 python -u tools/host_cost.py --camera $CAM --world $N --all-ranks --frames 300 > $O/all_ranks_${CAM}_N$N.log 2>&1; guard $? ranks-$CAM-$N $O/all_ranks_${CAM}_N$N.log
    grep "max over" $O/all_ranks_${CAM}_N$N.log
  done; done ;;
compact)  # slice-compacted duo boxes: parity, bound check, config-3 timing; rank-0 share replay; plane8
  timeout -k 10 900 $PYT tests/test_gpu_parity.py tests/test_gpu_baked.py tests/test_gpu_layout.py -k "duo or every_kernel_path or midsize or baked or plane" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  timeout -k 10 900 $PYT tests/test_gpu_fullsize.py -k "baked" > $O/pytest_full.log 2>&1; guard $? pytest $O/pytest_full.log
  tail -2 $O/pytest_full.log
  timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 1024x8 --baked --cameras C1,C0 --method 1 --rounds 5 --env "" "VR_PLANE8=0" > $O/variants_baked.log 2>&1; guard $? var $O/variants_baked.log
  grep -v "round\|amdgpu.ids" $O/variants_baked.log
  VRDD_LIB=tools/build/variants/boxcheck/libvr.so timeout -k 10 300 python -u tools/box_check.py > $O/box_check.log 2>&1; guard $? boxcheck $O/box_check.log
  tail -1 $O/box_check.log
  for M in 1 2; do
    timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method $M --rounds 5 --env "" "VR_DUO=0" "VR_DUO=3" "VR_DUO=4" > $O/variants_512x8_m$M.log 2>&1; guard $? var $O/variants_512x8_m$M.log
    grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
  done
  timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 256x4@512x512 --cameras C0 --method 1 --rounds 5 --env "" "VR_DUO=0" > $O/variants_256x4.log 2>&1; guard $? var $O/variants_256x4.log
  grep -v "round\|amdgpu.ids" $O/variants_256x4.log
  for CAM in C0 C1; do for N in 4 8; do
    timeout -k 10 300 python -u tools/host_cost.py --camera $CAM --world $N --all-ranks --frames 300 > $O/all_ranks_${CAM}_N$N.log 2>&1; guard $? ranks $O/all_ranks_${CAM}_N$N.log
    grep "max over" $O/all_ranks_${CAM}_N$N.log
  done; done ;;
dbg)  # the 512^3 C1 two-sample frame with and without slice compaction
  VRDD_LIB=tools/build/variants/boxcheck/libvr.so timeout -k 10 300 python -u tools/box_check.py --configs 512x8:C1,512x8:C0 --methods 1 --duos "VR_DUO=2+VR_DUO_COMPACT=0,2,3" > $O/box_check.log 2>&1
  grep -v amdgpu $O/box_check.log
  timeout -k 10 300 python -u tools/box_check.py --any-build --configs 512x8:C1 --methods 1 --duos "VR_DUO=2+VR_DUO_COMPACT=0,2" > $O/main.log 2>&1
  grep -v amdgpu $O/main.log ;;
sweep)  # baked C1 on the 8x2x2 copy: occupancy caps and ray splits; config 3 compaction / tile blocks
  timeout -k 10 600 python -u tools/bench_variants.py --variants main --config 1024x8 --baked --cameras C1 --method 1 --rounds 4 --env "" "VR_WG_PER_CU=3" "VR_WG_PER_CU=6" "VR_WG_PER_CU=8" "VR_SEG=-4" "VR_SEG=2" "VR_SEG=-2" "VR_SEG=8" > $O/variants_baked_C1.log 2>&1; guard $? var $O/variants_baked_C1.log
  grep -v "round\|amdgpu.ids" $O/variants_baked_C1.log
  timeout -k 10 600 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method 1 --rounds 6 --env "" "VR_DUO_COMPACT=0" "VR_XBLOCK=1,8" "VR_XBLOCK=2,4" "VR_XBLOCK=1,2" > $O/variants_512x8.log 2>&1; guard $? var $O/variants_512x8.log
  grep -v "round\|amdgpu.ids" $O/variants_512x8.log ;;
seg2)  # two segments per rank: GPU tests (gloo N = 2 chain, rehearsal), config 5 rehearsal
  timeout -k 10 900 $PYT tests/test_gpu_bench.py tests/test_gpu_gmm.py -k "gmm and not at_size" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  timeout -k 10 1000 python -u bench.py --config gmm2048 --slab-rehearsal --segments 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1; guard $? gmm5 $O/bench.log
  grep '^{' $O/bench.log | cut -c1-400 ;;
m3duo)  # entropy: several samples per slice-compacted box (no gap slices at 1024^3)
  for CFG in 1024x8 512x8; do
    timeout -k 10 600 python -u tools/bench_variants.py --variants main --config $CFG --cameras C0 --method 3 --rounds 3 --env "" "VR_PATH=1,VR_DUO=2,VR_DUO_COMPACT=1" "VR_PATH=1,VR_DUO=2,VR_DUO_COMPACT=1,VR_BOX_MAX=2048" "VR_PATH=1,VR_DUO=3,VR_DUO_COMPACT=1,VR_BOX_MAX=2048" "VR_PATH=1,VR_BOX_MAX=2048" > $O/variants_${CFG}_m3.log 2>&1; guard $? var $O/variants_${CFG}_m3.log
    grep -v "round\|amdgpu.ids" $O/variants_${CFG}_m3.log
  done ;;
wg)  # workgroup boxes (k_march_wgbox): parity, then config 3 / config 2 timing by rows and capacity
  timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "wgbox" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  for M in 1 2; do
    timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method $M --rounds 5 --env "" "VR_WG_ROWS=2" "VR_WG_ROWS=4" "VR_WG_ROWS=2,VR_BOX_WG=6144" "VR_WG_ROWS=4,VR_BOX_WG=6144" "VR_WG_ROWS=2,VR_WG_PER_CU=3" > $O/variants_512x8_m$M.log 2>&1; guard $? var $O/variants_512x8_m$M.log
    grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
  done
  timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 256x4@512x512 --cameras C0 --method 1 --rounds 5 --env "" "VR_WG_ROWS=2" "VR_WG_ROWS=4" > $O/variants_256x4.log 2>&1; guard $? var $O/variants_256x4.log
  grep -v "round\|amdgpu.ids" $O/variants_256x4.log ;;
wgpmc)  # fabric bytes per dispatch: per-wave duo vs workgroup boxes at 512^3 C0
  for E in "" "VR_WG_ROWS=2" "VR_WG_ROWS=4,VR_BOX_WG=6144"; do
    N=${E:-duo}; N=${N//[=,]/_}
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$N -o p -- python tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method 1 --rounds 1 --reps 3 --env "$E" > $O/pmc_$N.log 2>&1; guard $? pmc-$N $O/pmc_$N.log
    python tools/pmc_summary.py $O/pmc_$N "k_march_" | tee $O/pmc_$N.txt
  done ;;
wgp)  # workgroup boxes with the next box in flight (k_march_wgpipe): parity, timing, fabric bytes
  timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "wgbox" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  for M in 1 2; do
    timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method $M --rounds 5 --env "" "VR_WG_ROWS=2,VR_WG_PIPE=1" "VR_WG_ROWS=2,VR_WG_PIPE=1,VR_BOX_WG=1536" "VR_WG_ROWS=2,VR_WG_PIPE=1,VR_BOX_WG=6144" "VR_WG_ROWS=2,VR_WG_PIPE=1,VR_DUO=4,VR_BOX_WG=6144" "VR_WG_ROWS=2" > $O/variants_512x8_m$M.log 2>&1; guard $? var $O/variants_512x8_m$M.log
    grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
  done
  timeout -k 10 400 python -u tools/bench_variants.py --variants main --config 256x4@512x512 --cameras C0 --method 1 --rounds 5 --env "" "VR_WG_ROWS=2,VR_WG_PIPE=1" > $O/variants_256x4.log 2>&1; guard $? var $O/variants_256x4.log
  grep -v "round\|amdgpu.ids" $O/variants_256x4.log
  E="VR_WG_ROWS=2,VR_WG_PIPE=1"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_pipe -o p -- python tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method 1 --rounds 1 --reps 3 --env "$E" > $O/pmc_pipe.log 2>&1; guard $? pmc $O/pmc_pipe.log
  python tools/pmc_summary.py $O/pmc_pipe "k_march_" | tee $O/pmc_pipe.txt ;;
seg2b)  # config 5 rehearsal, two segments per rank, more balancing passes (the shortest period's cut kept)
  [ -n "$BENCH_ONLY" ] || { timeout -k 10 600 $PYT tests/test_gpu_bench.py -k "gmm" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log; tail -2 $O/pytest.log; }
  timeout -k 10 1100 python -u bench.py --config gmm2048 --slab-rehearsal --segments 2 --rebalance ${PASSES:-5} --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1; guard $? gmm5 $O/bench.log
  grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['period_ms_per_pass'], d['config']['kept_pass'], d['config']['rank_ms'])" ;;
cg)  # entropy workgroup boxes; direct-path corner batch 2 (variant cg2: fewer VGPRs in the box marches)
  timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "wgbox" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
  tail -2 $O/pytest.log
  timeout -k 10 600 python -u tools/bench_variants.py --variants main,cg2 --config 1024x8 --cameras C0 --method 3 --rounds 4 --env "" "VR_WG_ROWS=2" "VR_WG_ROWS=4" "VR_WG_ROWS=2,VR_BOX_WG=4096" > $O/variants_1024x8_m3.log 2>&1; guard $? var $O/variants_1024x8_m3.log
  grep -v "round\|amdgpu.ids" $O/variants_1024x8_m3.log
  for M in 1 2; do
    timeout -k 10 500 python -u tools/bench_variants.py --variants main,cg2 --config 512x8 --cameras C0 --method $M --rounds 5 --env "" > $O/variants_512x8_m$M.log 2>&1; guard $? var $O/variants_512x8_m$M.log
    grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
  done
  timeout -k 10 500 python -u tools/bench_variants.py --variants main,cg2 --config 512x8 --cameras C0 --method 3 --rounds 3 --env "" "VR_WG_ROWS=2" > $O/variants_512x8_m3.log 2>&1; guard $? var $O/variants_512x8_m3.log
  grep -v "round\|amdgpu.ids" $O/variants_512x8_m3.log
  timeout -k 10 400 python -u tools/bench_variants.py --variants main,cg2 --config 256x4@512x512 --cameras C0 --method 1 --rounds 5 --env "" > $O/variants_256x4.log 2>&1; guard $? var $O/variants_256x4.log
  grep -v "round\|amdgpu.ids" $O/variants_256x4.log ;;
gmm5k)  # config 5 rehearsal (two segments per rank) under rocprofv3 --kernel-trace --stats
  timeout -k 10 1100 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o gmm2048 -- python -u bench.py --config gmm2048 --slab-rehearsal --segments 2 --rebalance 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1; guard $? gmm5k $O/bench.log
  grep '^{' $O/bench.log | cut -c1-300 ;;
knobs)  # occupancy / samples-per-box sweep of configs 2 and 3 on the final build
  timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method 1 --rounds 4 --env "" "VR_WG_PER_CU=3" "VR_WG_PER_CU=5" "VR_WG_PER_CU=6" "VR_BOX_MAX=512" "VR_BOX_MAX=2048" "VR_NO_LPT=1" > $O/variants_512x8.log 2>&1; guard $? var $O/variants_512x8.log
  grep -v "round\|amdgpu.ids" $O/variants_512x8.log
  timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 256x4@512x512 --cameras C0 --method 1 --rounds 5 --env "" "VR_DUO=2" "VR_DUO=3" "VR_WG_PER_CU=2" "VR_WG_PER_CU=3" "VR_WG_PER_CU=6" "VR_XBLOCK=0" "VR_XBLOCK=1,1" > $O/variants_256x4.log 2>&1; guard $? var $O/variants_256x4.log
  grep -v "round\|amdgpu.ids" $O/variants_256x4.log
  timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 128x1@256x256 --cameras C0 --method 1 --rounds 5 --env "" "VR_SEG=-2" "VR_SEG=4" "VR_WG_PER_CU=2" "VR_XBLOCK=0" > $O/variants_128x1.log 2>&1; guard $? var $O/variants_128x1.log
  grep -v "round\|amdgpu.ids" $O/variants_128x1.log ;;
*) echo "unknown job $J"; exit 2 ;;
esac
echo done
