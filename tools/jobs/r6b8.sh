# round 6 (session 2): the codec march with 16x4 pixel blocks per wave (VR_CODEC_MAP=1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "codec" > $O/pytest_codec.log 2>&1 || { tail -30 $O/pytest_codec.log; exit 1; }
tail -1 $O/pytest_codec.log
for M in 4 5 6; do
timeout -k 10 400 python -u tools/bench_variants.py --codec --config 1024x8 --cameras C0,C1 --method $M --rounds 3 --reps 3 --env "" "VR_CODEC_MAP=1" > $O/codec_1024x8_m$M.log 2>&1 || exit 1
done
grep -E "median" $O/codec_*.log
echo ok
