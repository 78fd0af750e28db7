# round 6 (session 2): compact-block defaults (seg_map) against VR_SEG_MAP=0 on every launch kind they touch
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b7; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_baked.py > $O/pytest_parity_baked.log 2>&1 || { tail -30 $O/pytest_parity_baked.log; exit 1; }
tail -1 $O/pytest_parity_baked.log
V="python -u tools/bench_variants.py --rounds 5 --reps 5 --env VR_SEG_MAP=0 \"\""
timeout -k 10 300 python -u tools/bench_variants.py --rounds 5 --reps 5 --env "VR_SEG_MAP=0" "" --config 1024x8 --baked --cameras C0,C1 > $O/v_baked_1024x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --rounds 5 --reps 5 --env "VR_SEG_MAP=0" "" --config 512x8 --baked --cameras C0,C1 > $O/v_baked_512x8.log 2>&1 || exit 1
for M in 1 3; do
timeout -k 10 300 python -u tools/bench_variants.py --rounds 5 --reps 5 --env "VR_SEG_MAP=0" "" --config 128x1 --cameras C0,C1 --method $M > $O/v_128x1_m$M.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --rounds 5 --reps 5 --env "VR_SEG_MAP=0" "" --config 256x4 --cameras C0,C1 --method $M > $O/v_256x4_m$M.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/bench_variants.py --rounds 3 --reps 3 --env "VR_SEG_MAP=0" "" --config 1024x4@1920x1080 --cameras C0,C1 --method 3 > $O/v_1024x4_m3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --rounds 3 --reps 3 --env "VR_SEG_MAP=0" "" --config 1024x2@1920x1080 --cameras C0,C1 --method 3 > $O/v_1024x2_m3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --rounds 3 --reps 3 --env "VR_SEG_MAP=0" "" --config 1024x8 --cameras C0 --method 1 > $O/v_1024x8_m1.log 2>&1 || exit 1
grep -E "median" $O/v_*.log
echo ok
