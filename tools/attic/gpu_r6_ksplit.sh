#!/bin/bash
# Round 6: the fused forward's split-K narrow layers (FMLP_KSPLIT, build/libppomlp.so) against the
# one-wave-per-tile build (build/libppomlp_k0.so): the fused-PPO GPU tests, the captured update and
# rollout A/B, and 1000-iteration Go2 learning curves at 5 / 6 / 8 contact sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6_ksplit
mkdir -p $O
B=unitree-rl-gym_amd/csrc/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_ppo.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 2; }
tail -2 $O/tests.txt
rm -f gpurun_out/update_ab.log gpurun_out/update_ab_full.log
bash tools/gpu_update_ab.sh $B/libppomlp_k0.so $B/libppomlp.so > /dev/null || exit 3
cp gpurun_out/update_ab.log $O/update_ab.txt
bash tools/gpu_rollout_ab.sh $B/libppomlp_k0.so $B/libppomlp.so > /dev/null || exit 4
cp gpurun_out/rollout_ab.log $O/rollout_ab.txt
cat $O/update_ab.txt $O/rollout_ab.txt
for seed in 1 2; do
  for sw in 5 6 8; do
    timeout -k 10 200 python tools/learn_curve.py go2 1000 4096 - $sw $seed > $O/learn_go2_${sw}_seed$seed.log 2>&1 || exit 5
  done
done
for f in $O/learn_*.log; do echo $f; tail -n 1 $f; done
