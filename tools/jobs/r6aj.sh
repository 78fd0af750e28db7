# round 6: default-dispatch scan, codec volumes (methods 4/5/6) and 16/32-bin method 7, over views
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6aj; mkdir -p $O
for M in 4 5 6; do
timeout -k 10 400 python -u tools/bench_variants.py --codec --config 1024x8 --cameras C0,C1,S,T --method $M --rounds 2 --reps 2 > $O/codec_1024x8_m$M.log 2>&1 || exit 1
done
timeout -k 10 400 python -u tools/bench_variants.py --codec --config 512x8 --cameras C0,C1,S,T --method 6 --rounds 2 --reps 2 > $O/codec_512x8_m6.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x32@1920x1080 --cameras C0,C1,S,T --method 7 --rounds 2 --reps 2 > $O/m7_512x32.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x16@1920x1080 --cameras C0,C1,S,T --method 7 --rounds 2 --reps 2 > $O/m7_1024x16.log 2>&1 || exit 1
echo ok
