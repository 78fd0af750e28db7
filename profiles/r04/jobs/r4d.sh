#!/bin/bash
# round 4, job d: HW-queue sharing hypothesis for the N > 1 loop; baked side views on plane copies;
# rolled wide entropy; new and affected parity tests
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_baked.py tests/test_gpu_parity.py > $O/pytest_r4d.log 2>&1 || { tail -30 $O/pytest_r4d.log; exit 1; }
tail -2 $O/pytest_r4d.log
echo "GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES"
timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8_q4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 8 --priority -1 > $O/host_cost_N8_q4_prio.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8_q8.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8_q16.log 2>&1 || exit 1
for CAM in C0 S; do
timeout -k 10 400 python -u bench.py --config 1024x8 --camera $CAM --baked --no-cpu-baseline > $O/bench_baked_$CAM.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --config 1024x32 --method 3 --no-cpu-baseline > $O/bench_1024x32_C0_m3.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config 512x32 --method 3 --no-cpu-baseline > $O/bench_512x32_C0_m3.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config 512x8 --no-cpu-baseline > $O/bench_512x8_C0.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rank_sim.py --camera S --baked --worlds 2,4,8 --modes cost > $O/rank_sim_S_baked.log 2>&1 || exit 1
echo done
