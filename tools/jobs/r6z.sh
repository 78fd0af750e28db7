# round 6: side-view entropy (S, method 3): the axis-copy pipelined march vs the forced alternatives
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6z; mkdir -p $O
timeout -k 10 900 python -u tools/bench_variants.py --config 1024x8 --cameras S --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=0" "VR_PATH=4" > $O/side_m3.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras S --method 1 --rounds 3 > $O/side_m1.log 2>&1 || exit 1
echo ok
