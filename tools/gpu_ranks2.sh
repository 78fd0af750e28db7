cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
rm -f gpurun_out/ranks.log
for p in 4 0 1 3; do
  echo "VR_PATH=$p" >> gpurun_out/ranks.log
  VR_PATH=$p timeout -k 10 600 python -u tools/rank_sim.py --camera C0 >> gpurun_out/ranks.log 2>&1 || exit $?
done
