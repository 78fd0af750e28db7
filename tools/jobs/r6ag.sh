# round 6: wide records (16/32 bins) side / top / oblique views and narrow-record entropy: box march vs defaults
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ag; mkdir -p $O
for M in 1 3; do
timeout -k 10 500 python -u tools/bench_variants.py --config 1024x32@1920x1080 --cameras C1,S,T --method $M --rounds 2 --reps 2 --env "" "VR_PATH=1" > $O/wide_1024x32_m$M.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x16@1920x1080 --cameras C1,S --method $M --rounds 2 --reps 2 --env "" "VR_PATH=1" > $O/wide_1024x16_m$M.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x16@1920x1080 --cameras C1,S --method $M --rounds 2 --reps 2 --env "" "VR_PATH=1" > $O/wide_512x16_m$M.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/bench_variants.py --config 256x2@512x512 --cameras C0,C1,S --method 3 --rounds 2 --reps 3 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" > $O/m3_256x2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 384x4@768x768 --cameras C0,C1 --method 3 --rounds 2 --reps 3 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" > $O/m3_384x4.log 2>&1 || exit 1
echo ok
