#!/bin/bash
# H1 x 8192 (LSTM policy) PPO iteration: collection / update split, then per-kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=${1:-h1}; N=${2:-8192}
timeout -k 10 300 python tools/ppo_breakdown.py $T $N 3 > gpurun_out/${T}_breakdown.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}prof -o run --output-format csv -- python tools/ppo_breakdown.py $T $N 3 > gpurun_out/${T}prof.log 2>&1 || exit 3
find gpurun_out/${T}prof -name "*kernel_trace.csv" -delete
tail -1 gpurun_out/${T}_breakdown.log
python tools/kernel_stats_top.py gpurun_out/${T}prof 30
