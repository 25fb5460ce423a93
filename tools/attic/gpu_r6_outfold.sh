#!/bin/bash
# Round 6: the output layer's backward folded into the forward + loss launch and the first
# layer's weight-gradient launch (PMLP_OUT_FOLD, default on) -- the fused-PPO GPU tests, the
# captured update A/B against PMLP_OUT_FOLD=0 (its own pair launch), and the cross-physics
# policy evaluation of the sweep-count study.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6_outfold
mkdir -p $O
B=unitree-rl-gym_amd/csrc/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_training_drift.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 2; }
tail -2 $O/tests.txt
rm -f gpurun_out/update_ab.log gpurun_out/update_ab_full.log
A_ENV='PMLP_OUT_FOLD=0' bash tools/gpu_update_ab.sh $B/libppomlp.so $B/libppomlp.so > /dev/null || exit 3
cp gpurun_out/update_ab.log $O/update_ab.txt
cat $O/update_ab.txt
timeout -k 10 300 python tools/probes/sweeps_policy_eval.py 8 300 500 5 8 > $O/policy_eval_train8.txt 2>&1 || exit 4
timeout -k 10 300 python tools/probes/sweeps_policy_eval.py 5 300 500 5 8 > $O/policy_eval_train5.txt 2>&1 || exit 5
grep -h trained $O/policy_eval_*.txt
