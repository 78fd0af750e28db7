# round 6: default-dispatch scan, small configs and 32-bin records (views x methods)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ae; mkdir -p $O
for M in 1 2 3 7; do
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1,S,T --method $M --rounds 2 --reps 3 > $O/scan_256x4_m$M.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 128x1 --cameras C0,C1,S,T --method $M --rounds 2 --reps 3 > $O/scan_128x1_m$M.log 2>&1 || exit 1
done
for M in 1 3; do
timeout -k 10 400 python -u tools/bench_variants.py --config 512x32@1920x1080 --cameras C0,C1,S,T --method $M --rounds 2 --reps 2 > $O/scan_512x32_m$M.log 2>&1 || exit 1
done
echo ok
