# round 6: k_march_pair (two rays per lane) -- parity, then timing against the duo / k_march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "pair or every_kernel_path" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0,C1 --rounds 5 --env '' VR_PAIR=1,VR_PATH=1 VR_DUO=0,VR_PATH=1 VR_PAIR=1,VR_PATH=1,VR_WG_PER_CU=4 > $O/var_512x8.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 512x8 --cameras C0 --method 2 --rounds 5 --env '' VR_PAIR=1,VR_PATH=1 > $O/var_512x8_m2.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 256x4 --cameras C0 --rounds 5 --env '' VR_PAIR=1,VR_PATH=1 VR_DUO=2 > $O/var_256x4.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/bench_variants.py --variants main --config 1024x8 --cameras C0 --rounds 3 --env '' VR_PAIR=1,VR_PATH=1 VR_DUO=0,VR_PATH=1 > $O/var_1024x8.log 2>&1 || exit 1
echo ok
