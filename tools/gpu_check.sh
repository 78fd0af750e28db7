cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config 256x4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_256.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config 1024x8 --steps 10 --warmup 2 > gpurun_out/bench_1024.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r01 -- python bench.py --config 1024x8 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
echo done
