#!/bin/bash
# GMM refill vs lockstep batches, 512^3 x K16; FETCH_SIZE per variant.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/gmm2; mkdir -p $O
for LS in 0 1; do
  VR_GMM_LOCKSTEP=$LS timeout -k 10 120 python -u tools/gmm_time.py --dim 512 > $O/t_ls$LS.log 2>&1 || { cat $O/t_ls$LS.log; exit 1; }
  echo "lockstep=$LS"; grep -v amdgpu.ids $O/t_ls$LS.log
  VR_GMM_LOCKSTEP=$LS timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$LS -o f -- python tools/gmm_time.py --dim 512 --cams C0 --methods 1 --reps 3 > $O/f$LS.log 2>&1 || { tail $O/f$LS.log; exit 1; }
  python3 tools/pmc_summary.py $O/f$LS "16, 1, false>"
done
