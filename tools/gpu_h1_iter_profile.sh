#!/bin/bash
# kernel trace of H1 x 8192 PPO iterations (LSTM policy) and the iteration breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/h1iter
rm -rf $O && mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python tools/ppo_breakdown.py ${1:-h1} ${2:-8192} 3 > $O/run.log 2>&1 || exit 2
python tools/iter_trace.py $O/tr/run_kernel_trace.csv > $O/iteration_breakdown.txt 2>&1 || exit 3
find $O -name "*kernel_trace.csv" -delete
head -40 $O/iteration_breakdown.txt
