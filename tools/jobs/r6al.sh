# round 6: register-decoded entropy (pipelined / segmented marches): series log (main) vs the table form from constant memory (ctab)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6al; mkdir -p $O
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1,S --method 3 --rounds 3 --reps 3 > $O/ctab_256x4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 128x1 --cameras C0,C1 --method 3 --rounds 3 --reps 3 > $O/ctab_128x1.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x2@1920x1080 --cameras C0,C1 --method 3 --rounds 2 --reps 2 > $O/ctab_1024x2.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x4@1920x1080 --cameras C0,C1,S --method 3 --rounds 2 --reps 2 > $O/ctab_1024x4.log 2>&1 || exit 1
echo ok
