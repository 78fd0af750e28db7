# round 6: oblique entropy at 1024^3 x 8 after the four-bin chunks: quad march vs LDS box
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ar; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C1 --method 3 --rounds 3 --reps 2 --env "" "VR_PATH=1" "VR_PATH=7" "VR_WG_PER_CU=3" "VR_WG_PER_CU=1" > $O/c1_m3_paths.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x16@1920x1080 --cameras C1 --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=1" > $O/c1_m3_x16.log 2>&1 || exit 1
echo ok
