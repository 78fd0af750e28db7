#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/warm; mkdir -p $O
for A in "" "--baked" "--camera C1 --no-cpu-baseline" "--baked --camera C1 --no-cpu-baseline"; do
timeout -k 10 300 python bench.py --no-cpu-baseline $A --warmup 5 > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('bench $A', d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])"
done
timeout -k 10 300 python bench.py --config gmm96 --no-cpu-baseline > $O/g.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/g.json'));print('bench gmm96', d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])"
