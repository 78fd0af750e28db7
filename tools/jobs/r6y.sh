# round 6: frame-order knobs for the headline frame (1024^3 x 8, C0, method 1), one process
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 900 python -u tools/bench_variants.py --config 1024x8 --cameras C0 --method 1 --rounds 4 --env "" "VR_XBLOCK=1,8" "VR_XBLOCK=2,4" "VR_XBLOCK=1,2" "VR_XBLOCK=2,8" "VR_XBLOCK=1,16" "VR_NO_LPT=1" "VR_NO_ADAPT=1" "VR_WG_PER_CU=6" "VR_WG_PER_CU=4" > $O/knobs_C0.log 2>&1 || exit 1
echo ok
