#!/bin/bash
# round 4, job z: two samples per box with the second sample's planes decoded after the
# first sample (k_march_duo<.., SPLIT>) -- parity, timing, traffic
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "duo or every_kernel_path or coarse" > $O/pytest_r4z.log 2>&1 || { tail -30 $O/pytest_r4z.log; exit 1; }
tail -1 $O/pytest_r4z.log
for M in 1 2; do
  timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method $M --rounds 5 --env "VR_DUO=0" "" "VR_DUO=5" > $O/variants_512x8_m$M.log 2>&1 || exit 1
  grep -v "round\|amdgpu.ids" $O/variants_512x8_m$M.log
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/$C -o p -- python tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 2 --reps 2 --env "VR_DUO=0" "" "VR_DUO=5" > $O/pmc_$C.log 2>&1 || { tail -20 $O/pmc_$C.log; exit 1; }
done
python tools/rank_pmc.py $O/FETCH_SIZE/p_counter_collection.csv $O/WRITE_SIZE/p_counter_collection.csv > $O/pmc_split.log || exit 1
cat $O/pmc_split.log
echo done
