#!/bin/bash
# fused PPO kernels: parity tests, then the optimizer-step timing and per-kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_ppo.py tests/test_gpu_env.py -k "fused or rollout" > gpurun_out/upd_tests.log 2>&1
rc=$?; tail -2 gpurun_out/upd_tests.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/updprof -o run --output-format csv -- python tools/probes/update_step_time.py > gpurun_out/upd_time.log 2>&1 || exit 3
grep TOTAL gpurun_out/upd_time.log
find gpurun_out/updprof -name "*kernel_trace.csv" -delete
python tools/kernel_stats_top.py gpurun_out/updprof 14
