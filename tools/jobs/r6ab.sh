# round 6: default-dispatch scan over views x methods (looking for pathological choices)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ab; mkdir -p $O
for M in 1 2 3 7; do
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1,S,T --method $M --rounds 2 --reps 2 > $O/scan_1024x8_m$M.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1,S,T --method $M --rounds 2 --reps 2 > $O/scan_512x8_m$M.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1,S,T --method 1 --baked --rounds 2 --reps 2 > $O/scan_1024x8_baked_m1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1,S,T --method 3 --baked --rounds 2 --reps 2 > $O/scan_1024x8_baked_m3.log 2>&1 || exit 1
echo ok
