#!/bin/bash
# Round-3: z-rows copy for side views -- parity tests, rotation sweep with and without it.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3e}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -30 $3; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -rf --timeout 300 --timeout-method thread -k "axis_views or full_frame or kernel_path or environment" > $O/pytest.log 2>&1; guard $? pytest $O/pytest.log
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/rot_sweep.py --rx 0,90 --step 10 > $O/rot_sweep.log 2>&1; guard $? rot $O/rot_sweep.log
grep -v amdgpu $O/rot_sweep.log
echo done
