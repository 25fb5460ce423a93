#!/bin/bash
# PPO loss step: the quad-per-row kernel (k_ppo_loss_step_q) vs the one-lane-per-row kernel
# (PMLP_LOSS_QUAD=0), kernel-trace stats of the eager optimizer-step probe; parity test first
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/loss_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_ppo.py -v --timeout 120 --timeout-method thread \
    -k "loss_step_kernel or matches_fp32_autograd_update or graph_is_bitwise" > $O/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|^E  " $O/tests.log | head -30; [ $rc -eq 0 ] || exit 2
for q in 1 0 1 0; do
  PMLP_LOSS_QUAD=$q timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/q$q -o run --output-format csv \
      -- python tools/probes/update_step_time.py > $O/q$q.log 2>&1 || exit 3
  echo "== PMLP_LOSS_QUAD=$q"; python tools/kernel_stats_top.py $O/q$q 40 | grep -E "loss|total"
  rm -rf $O/q$q
done
