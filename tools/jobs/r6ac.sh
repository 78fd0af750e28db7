# round 6: side / top views of the coarse 512^3 x 8 volume (methods 1, 2) and method 7 side views: forced alternatives
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ac; mkdir -p $O
for M in 1 2; do
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras S,T --method $M --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=1,VR_DUO=2" "VR_PATH=7" "VR_PATH=0" "VR_ZROWS=0" > $O/side_512x8_m$M.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras S,T --method 7 --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" "VR_PATH=0" > $O/side_1024x8_m7.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras S,C1 --method 7 --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=7" "VR_PATH=0" > $O/side_512x8_m7.log 2>&1 || exit 1
echo ok
