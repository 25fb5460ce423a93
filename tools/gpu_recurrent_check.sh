#!/bin/bash
# recurrent PPO: parity tests (+ the fused-loss PPO tests), then the H1 x 8192 iteration
# breakdown with kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_recurrent.py tests/test_gpu_fused_ppo.py > gpurun_out/rec_tests.log 2>&1
rc=$?; tail -5 gpurun_out/rec_tests.log; [ $rc -eq 0 ] || exit 2
bash tools/gpu_h1_breakdown.sh h1 8192
