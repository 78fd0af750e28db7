#!/bin/bash
# PMC traffic per launch of one bench.py workload (3 separate passes).
# usage: bash tools/gpu_pmc1.sh KEY OUTDIR -- <bench.py args>
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
KEY=$1; O=gpurun_out/$2; shift 3
mkdir -p $O
i=0
for CTRS in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $CTRS --output-format csv -d $O/p$i -o p$i -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" > $O/p$i.log 2>&1 || exit $?
done
python tools/pmc_traffic.py $O/traffic.json "$KEY" $O/p1.log $O/p1 $O/p2 $O/p3 > /dev/null || exit 1
python -c "
import json; d=json.load(open('$O/traffic.json'))
for k,v in d.items(): print(k, round(v['hbm_bytes_per_launch']/1e9,3), 'GB', v.get('kernel'))"
grep -o '"kernel_ms": [0-9.]*' $O/p1.log
