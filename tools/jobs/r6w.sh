# round 6: entropy terms in chunks of 2 (main) / 4 / 8 bins vs the committed build (prev)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 5 > $O/ab_m3_1024x8.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 3 --rounds 5 > $O/ab_m3_512x8.log 2>&1 || exit 1
echo ok
