# round 6: paired branch-free entropy terms (main) vs the committed build (prev)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 6 > $O/ab_m3_1024x8.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 3 --rounds 6 > $O/ab_m3_512x8.log 2>&1 || exit 1
echo ok
