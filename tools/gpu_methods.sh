cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
for m in 2 3 7; do
  timeout -k 10 600 python -u tools/bench_variants.py --rounds 2 --method $m --env "" VR_PATH=0 VR_PATH=2 VR_PATH=1 >> gpurun_out/methods.log 2>> gpurun_out/methods.err || exit $?
done
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --rounds 3 --env "" VR_PATH=1 VR_PATH=4 >> gpurun_out/methods.log 2>> gpurun_out/methods.err || exit $?
