#!/bin/bash
# Fused-PPO parity tests, then kernel-trace stats of the eager optimizer-step probe for the
# small reduction / optimizer kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/small_k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_ppo.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv \
    -- python tools/probes/update_step_time.py > $O/t.log 2>&1 || exit 3
python tools/kernel_stats_top.py $O/t 40 | grep -E "k_opt_prepare|k_ppo_loss|k_adam|k_reduce"
rm -rf $O/t
