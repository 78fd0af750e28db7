#!/bin/bash
# Baked statistics (basicDataProcessing): parity tests, path sweep, bench lines
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_baked.py tests/test_gpu_parity.py -k "baked or isabel or codec_via" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for C in 1024x8 512x8; do
timeout -k 10 400 python -u tools/bench_variants.py --baked --config $C --rounds 3 --method 1 --cameras C0,C1 --env "" "VR_PATH=1" "VR_PATH=7,VR_SEG=-2" "VR_PATH=7,VR_SEG=-4" "VR_PATH=7,VR_SEG=2" "VR_PATH=7,VR_SEG=4" "VR_WG_PER_CU=4" > $O/var_$C.log 2>&1 || { tail -20 $O/var_$C.log; exit 1; }
grep -v "round\|amdgpu" $O/var_$C.log
done
timeout -k 10 300 python -u bench.py --baked --no-cpu-baseline > $O/bench_1024x8_C0_baked.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench_1024x8_C0_baked.json
