#!/bin/bash
# Round-3: axis views at 512^3 (copy vs the coarse-volume segmented march), LDS-box march for wide records at 1024^3.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3f}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "axis_views or full_frame or kernel_path or environment or random or coarse" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/rot_sweep.py --config 512x8 --rx 0 --step 10 --paths 7 > $O/rot_sweep_512.log 2>&1; guard $? rot $O/rot_sweep_512.log
grep -v amdgpu $O/rot_sweep_512.log
for CFG in 1024x32 1024x16; do
  timeout -k 10 400 python -u tools/bench_variants.py --config $CFG --rounds 2 --reps 3 --method 1 --env "" "VR_PATH=1" > $O/wide_box_$CFG.log 2>&1; guard $? wide-$CFG $O/wide_box_$CFG.log
  grep -v "round\|amdgpu" $O/wide_box_$CFG.log
done
echo done
