#!/bin/bash
# Kernel trace of bench.py itself (Go2 4096, 5 timed PPO iterations) and the iteration
# breakdown (collection / update phases, per-kernel totals, idle gaps) from it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/iterprof
rm -rf $O && mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no_cpu_baseline --no_other_configs > $O/bench.log 2>&1 || exit 7
python tools/iter_trace.py $O/bench/run_kernel_trace.csv > $O/iteration_breakdown.txt 2>&1 || exit 8
find $O -name "*kernel_trace.csv" -delete
head -50 $O/iteration_breakdown.txt
