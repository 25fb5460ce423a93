#!/bin/bash
# kernel sequence of one H1 x 8192 recurrent optimizer step
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/h1trace -o run --output-format csv -- python tools/ppo_breakdown.py h1 8192 2 > gpurun_out/h1trace.log 2>&1 || exit 2
python tools/step_kernels.py $(find gpurun_out/h1trace -name "*kernel_trace.csv" | head -1) > gpurun_out/h1_step_kernels.txt || exit 3
find gpurun_out/h1trace -name "*kernel_trace.csv" -delete
tail -3 gpurun_out/h1_step_kernels.txt
