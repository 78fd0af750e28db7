# round 6: entropy of narrow records (1-4 bins, configs 1-2) and 32-bin oblique / side views: kernels and forced alternatives
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6af; mkdir -p $O
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1,S --method 3 --rounds 2 --reps 3 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" "VR_PATH=4" "VR_PATH=0" > $O/m3_256x4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 128x1 --cameras C0,C1 --method 3 --rounds 2 --reps 3 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" "VR_PATH=4" > $O/m3_128x1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1,S --method 1 --rounds 2 --reps 3 > $O/m1_256x4.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x32@1920x1080 --cameras C1,S --method 1 --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" > $O/m1_512x32.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x32@1920x1080 --cameras C1,S --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" > $O/m3_512x32.log 2>&1 || exit 1
echo ok
