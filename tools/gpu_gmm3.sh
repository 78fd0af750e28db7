#!/bin/bash
# GMM at 1024^3 x K16 (206 GB resident) and 768^3: refill vs lockstep.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/gmm3; mkdir -p $O
for D in 768 1024; do for LS in 0 1; do
  VR_GMM_LOCKSTEP=$LS timeout -k 10 200 python -u tools/gmm_time.py --dim $D --reps 5 > $O/t${D}_ls$LS.log 2>&1 || { cat $O/t${D}_ls$LS.log; exit 1; }
  echo "dim=$D lockstep=$LS"; grep -v amdgpu.ids $O/t${D}_ls$LS.log
done; done
