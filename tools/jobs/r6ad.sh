# round 6: coarse side / top views on the box duo march -- tests, timing; coarse oblique alternatives
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_baked.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "512x8" > $O/pytest_fullsize_512.log 2>&1 || exit 1
for M in 1 2; do
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras S,T,C1 --method $M --rounds 2 --reps 2 --env "" "VR_PATH=1,VR_DUO=2" "VR_PATH=1" > $O/coarse_512x8_m$M.log 2>&1 || exit 1
done
echo ok
