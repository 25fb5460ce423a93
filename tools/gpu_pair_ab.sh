#!/bin/bash
# Paired backward GEMMs: the bitwise test and the fused-PPO suite, then the captured-update A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pair_ab
mkdir -p $O
bash tools/gpu_tests.sh tests/test_gpu_fused_ppo.py -x; rc=$?; cp gpurun_out/tests.log $O/tests.txt; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python tools/probes/update_pair_ab.py > $O/update_ab.txt 2>&1 || exit 3
cat $O/update_ab.txt
