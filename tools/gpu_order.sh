#!/bin/bash
# Full-frame dispatch order: longest-first per XCD (default) vs raster block order
# per XCD (VR_NO_LPT: neighbouring blocks, on different XCDs, run at the same time
# and depth, so lines they share can meet in the Infinity Cache), block shapes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x8 --rounds 5 --reps 5 \
  --env '' 'VR_NO_LPT=1' 'VR_NO_LPT=1,VR_XBLOCK=1,1' 'VR_NO_LPT=1,VR_XBLOCK=2,2' \
        'VR_NO_LPT=1,VR_XBLOCK=1,8' 'VR_NO_ADAPT=1' > gpurun_out/order.log 2>&1 || { tail -20 gpurun_out/order.log; exit 1; }
grep -v "^round" gpurun_out/order.log
