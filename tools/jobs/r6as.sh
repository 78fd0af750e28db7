# round 6: entropy log ablation on the final build (timing bound only; the nolog build is NOT exact)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6as; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 3 --reps 2 > $O/ablate_final_m3_1024x8.log 2>&1 || exit 1
echo ok
