# round 6: exact-log reductions side by side (193 centres on frexp vs 257 bit-space centres) against the committed build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 6 > $O/ab_m3_1024x8.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 3 --rounds 6 > $O/ab_m3_512x8.log 2>&1 || exit 1
echo ok
