# round 6: GMM error paths (2^23-pixel slab limit); config-5 rehearsal repeated
# twice (reproducibility of the kept cut and of the period estimate)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gmm.py -x -q -k errors --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 600 python -u bench.py --config gmm2048 --slab-rehearsal --segments 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/rehearsal_$i.log 2>&1 || exit 1
done
echo ok
