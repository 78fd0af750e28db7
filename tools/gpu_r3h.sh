#!/bin/bash
# Round-3: LDS-box march (16x4 wave blocks, now its default) vs the default dispatch for wide records and entropy.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3h}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "kernel_path or coarse or wide or random" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
tail -1 $O/pytest.log
for CM in 1024x32:1 1024x32:2 1024x32:3 1024x16:3 1024x16:2 512x32:1 512x32:3 512x8:3 1024x8:3; do
  CFG=${CM%%:*}; M=${CM#*:}
  timeout -k 10 400 python -u tools/bench_variants.py --config $CFG --rounds 2 --reps 3 --method $M --cameras C0 --env "" "VR_PATH=1" > $O/box_${CFG}_m$M.log 2>&1; guard $? box-$CM $O/box_${CFG}_m$M.log
  grep -v "round\|amdgpu" $O/box_${CFG}_m$M.log
done
echo done
