# round 6 session 3: per-rank PMC traffic of the N = 2/4/8 headline splits on the HEAD build
# (tools/rank_traffic.py), the N = 2 gloo line reading it, then config 3 and config 2 rounds
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6f2; mkdir -p $O
cp profiles/traffic.json $O/traffic.json
for N in 2 4 8; do
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/rt$N/f -o f -- python tools/rank_traffic.py run --world $N > $O/rt${N}_run.json 2> $O/rt${N}_f.log || { echo "fetch pass N=$N failed"; tail -5 $O/rt${N}_f.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/rt$N/w -o w -- python tools/rank_traffic.py run --world $N > $O/rt${N}_run_w.json 2> $O/rt${N}_w.log || { echo "write pass N=$N failed"; tail -5 $O/rt${N}_w.log; exit 1; }
  PMC_TAG=r6f2 python tools/rank_traffic.py fold $O/traffic.json $O/rt${N}_run.json $O/rt$N/f $O/rt$N/w > $O/rt${N}_fold.log 2>&1 || { cat $O/rt${N}_fold.log; exit 1; }
done
timeout -k 10 900 python -u bench.py --gpus 2 --dist-backend gloo --traffic-json $O/traffic.json > $O/bench_n2_traffic.log 2>&1 || exit 1
cp $O/traffic.json $O/traffic_ranks.json
RANKSIM=0 bash tools/gpu_round.sh r6f2 512x8:C0 256x4:C0 || exit 1
echo ok
