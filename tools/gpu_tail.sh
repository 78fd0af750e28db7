#!/bin/bash
# baked C0: bench.py vs bench_variants timing difference (adaptive order? zeroing?)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/tail; mkdir -p $O
for E in "" "VR_NO_ADAPT=1"; do
env $E timeout -k 10 300 python bench.py --baked --no-cpu-baseline > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('bench baked C0 env=$E', d['ms_per_step'], d['roofline']['kernel_ms'])"
env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('$O/b.json'));print('bench per-step C0 env=$E', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u tools/bench_variants.py --baked --config 1024x8 --rounds 3 --method 1 --cameras C0 --env "" "VR_NO_ADAPT=1" > $O/v.log 2>&1 || exit 1
grep -v "round\|amdgpu" $O/v.log
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --rounds 3 --method 1 --cameras C0 --env "" "VR_NO_ADAPT=1" > $O/v2.log 2>&1 || exit 1
grep -v "round\|amdgpu" $O/v2.log
