# round 6: codec marches -- quad vs lane-per-ray on oblique / side views, and method 7 wide on the lane-owned march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ak; mkdir -p $O
for M in 4 6; do
timeout -k 10 400 python -u tools/bench_variants.py --codec --config 1024x8 --cameras C1,S --method $M --rounds 2 --reps 2 --env "" "VR_CODEC_QUAD=0" > $O/codec_1024x8_m${M}_quad.log 2>&1 || exit 1
done
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x16@1920x1080 --cameras C1,S --method 7 --rounds 2 --reps 2 --env "" "VR_M7_WQ=0" > $O/m7_1024x16_wq.log 2>&1 || exit 1
echo ok
