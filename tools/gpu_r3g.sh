#!/bin/bash
# Round-3: the LDS-box march with 16x4-pixel wave blocks (VR_BOX_MAP=1) vs its 64x1 rows and the default kernels.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3g}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "kernel_path or coarse" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
tail -1 $O/pytest.log
for CFG in 512x8 1024x8 1024x16 1024x32; do
  timeout -k 10 400 python -u tools/bench_variants.py --config $CFG --rounds 2 --reps 3 --method 1 --cameras C0 --env "" "VR_PATH=1" "VR_PATH=1,VR_BOX_MAP=1" > $O/box_$CFG.log 2>&1; guard $? box-$CFG $O/box_$CFG.log
  grep -v "round\|amdgpu" $O/box_$CFG.log
done
timeout -k 10 400 python -u tools/bench_variants.py --config 512x8 --rounds 2 --reps 3 --method 2 --cameras C0 --env "" "VR_BOX_MAP=1" > $O/box_512x8_m2.log 2>&1; guard $? box-m2 $O/box_512x8_m2.log
grep -v "round\|amdgpu" $O/box_512x8_m2.log
echo done
