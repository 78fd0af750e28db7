# round 6: kernel choice for the oblique entropy frame (C1, method 3) after the cheaper log
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C1 --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=4" "VR_PATH=2" > $O/path_m3_C1.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0 --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=4" "VR_PATH=0" > $O/path_m3_C0.log 2>&1 || exit 1
echo ok
