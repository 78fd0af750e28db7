# round 6 (session 2): VR_SEG_MAP=1 on the headline march, side views and the N-rank tile lists
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b6; mkdir -p $O
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x8 --cameras C0,S --method 1 --rounds 5 --reps 5 --env "" "VR_SEG_MAP=1" > $O/map_1024x8_m1.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x8 --cameras C0,S --method 2 --rounds 3 --reps 3 --env "" "VR_SEG_MAP=1" > $O/map_1024x8_m2.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x4@1920x1080 --cameras C0,C1 --method 3 --rounds 3 --reps 3 --env "" "VR_SEG_MAP=1" > $O/map_1024x4_m3.log 2>&1 || exit 1
grep -E "median" $O/map_*.log
for CAM in C0 C1; do
  timeout -k 10 400 python -u tools/rank_sim.py --camera $CAM --modes cost --worlds 2,4,8 --envs "" "VR_SEG_MAP=1" > $O/rank_sim_$CAM.log 2>&1 || { tail $O/rank_sim_$CAM.log; exit 1; }
  timeout -k 10 400 python -u tools/rank_sim.py --camera $CAM --baked --modes cost --worlds 2,4,8 --envs "" "VR_SEG_MAP=1" > $O/rank_sim_baked_$CAM.log 2>&1 || { tail $O/rank_sim_baked_$CAM.log; exit 1; }
done
tail -n 12 $O/rank_sim_*.log
echo ok
