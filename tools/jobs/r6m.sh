# round 6: entropy decode ablation on the 193-centre log build (timing bound only; ablated builds are NOT exact)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 4 > $O/ablate_m3_1024x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0 --method 1 --rounds 3 --variants main > $O/m1_1024x8.log 2>&1 || exit 1
echo ok
