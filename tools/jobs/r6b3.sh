# round 6 (session 2): k_march_duop (unconditional prefetch loads
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "duo_march_early_exit" > $O/pytest_duo.log 2>&1 || { tail -30 $O/pytest_duo.log; exit 1; }
tail -1 $O/pytest_duo.log
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras C0,S --method 1 --rounds 5 --reps 5 --env "" "VR_DUOP=1" "VR_DUOP=1,VR_LOCK=1" "VR_DUOP=1,VR_LOCK=2" > $O/duop_512x8_m1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method 2 --rounds 5 --reps 5 --env "" "VR_DUOP=1" "VR_DUOP=1,VR_LOCK=1" "VR_DUOP=1,VR_LOCK=2" > $O/duop_512x8_m2.log 2>&1 || exit 1
grep -E "median" $O/duop_*.log
for L in 0 1 2; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_l$L -o f -- python tools/pmc_frames.py --config 512x8 --camera C0 --method 1 --tune VR_DUOP=1 VR_LOCK=$L --frames 3 > $O/pmc_l$L.log 2>&1 || { tail $O/pmc_l$L.log; exit 1; }
  grep identical $O/pmc_l$L.log
done
echo ok
