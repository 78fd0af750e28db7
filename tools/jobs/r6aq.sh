# round 6: frame-order block shapes for config 3 (512^3 x 8, 1080p, C0, method 1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6aq; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 4 --reps 3 --env "" "VR_XBLOCK=2,2" "VR_XBLOCK=1,1" "VR_XBLOCK=1,2" "VR_XBLOCK=2,1" "VR_XBLOCK=4,1" "VR_XBLOCK=4,2" "VR_XBLOCK=3,2" "VR_XBLOCK=2,3" "VR_XBLOCK=8,1" "VR_XBLOCK=8,2" > $O/xblock_512x8_C0_small.log 2>&1 || exit 1
echo ok
