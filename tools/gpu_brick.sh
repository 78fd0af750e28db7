#!/bin/bash
# 2x2 (x, y) micro-brick copy for the quad marches (oblique views): parity tests,
# interleaved A/B kernel ms (VR_BRICK=0 = x rows) at C1 for the methods given
# (default 1 2 3 7), PMC traffic per launch of the method-1 brick march at C1.
# usage: bash tools/gpu_brick.sh [methods...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/brick && export TMPDIR=/tmp
O=gpurun_out/brick
METHODS=${@:-1 2 3 7}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "brick or every_kernel_path or small_scene or method7" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for M in $METHODS; do
  timeout -k 10 300 python -u tools/bench_variants.py --rounds 5 --reps 5 --cameras C1 --method $M --env '' 'VR_BRICK=0' > $O/ab_m$M.log 2>&1 || exit $?
  tail -2 $O/ab_m$M.log
done
i=0
for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc_C1/p$i -o p$i -- python bench.py --camera C1 --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_C1_p$i.log 2>&1 || exit $?
done
python tools/pmc_traffic.py $O/traffic.json "1024x8|C1|m1" $O/pmc_C1_p1.log $O/pmc_C1/p1 $O/pmc_C1/p2 $O/pmc_C1/p3 > /dev/null || exit 1
python -c "
import json; d=json.load(open('$O/traffic.json'))
for k,v in d.items(): print(k, round(v['hbm_bytes_per_launch']/1e9,3), 'GB', v.get('kernel'))"
