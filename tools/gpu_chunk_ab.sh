#!/bin/bash
# recurrent update: row-chunk size of the split weight gradients (MLP heads, LSTM)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_recurrent.py tests/test_gpu_fused_ppo.py > gpurun_out/rec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rec_tests.log; [ $rc -eq 0 ] || exit 2
for cfg in "SPLITK_CHUNK=4096 LSTM_ROWS_CHUNK=2048" "SPLITK_CHUNK=1024 LSTM_ROWS_CHUNK=2048" "SPLITK_CHUNK=512 LSTM_ROWS_CHUNK=2048" "SPLITK_CHUNK=512 LSTM_ROWS_CHUNK=512" "SPLITK_CHUNK=512 LSTM_ROWS_CHUNK=1024"; do
  echo "== $cfg"; env $cfg timeout -k 10 300 python tools/ppo_breakdown.py h1 8192 3 2>&1 | tail -1 || exit 3
done
