# round 6 (session 2): pipelined march with its tile's waves paced within D steps (VR_LOCK=D) on the headline frame
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "every_kernel_path" > $O/pytest_pace.log 2>&1 || { tail -30 $O/pytest_pace.log; exit 1; }
tail -1 $O/pytest_pace.log
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x8 --cameras C0 --method 1 --rounds 5 --reps 5 --env "" "VR_LOCK=2" "VR_LOCK=4" "VR_LOCK=8" > $O/pace_1024x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 5 --reps 5 --env "" "VR_LOCK=4" "VR_LOCK=8" > $O/pace_512x8.log 2>&1 || exit 1
grep -E "median" $O/pace_*.log
for L in 0 2 4 8; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_l$L -o f -- python tools/pmc_frames.py --config 1024x8 --camera C0 --method 1 --tune VR_LOCK=$L --frames 3 > $O/pmc_l$L.log 2>&1 || { tail $O/pmc_l$L.log; exit 1; }
  grep identical $O/pmc_l$L.log
done
for L in 0 4 8; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc512_l$L -o f -- python tools/pmc_frames.py --config 512x8 --camera C0 --method 1 --tune VR_LOCK=$L --frames 3 > $O/pmc512_l$L.log 2>&1 || { tail $O/pmc512_l$L.log; exit 1; }
  grep identical $O/pmc512_l$L.log
done
echo ok
