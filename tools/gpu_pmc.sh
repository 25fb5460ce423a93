# k_step kernel trace + separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md HBM recipe)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python tools/profile_env.py go2 4096 100 > gpurun_out/prof_trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > gpurun_out/prof_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > gpurun_out/prof_write.log 2>&1 || exit 4
python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write k_step gpurun_out/pmc_k_step.json
