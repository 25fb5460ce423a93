set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_mlp4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mlp4 -o run --output-format csv -- python tools/probes/mlp4_time.py > gpurun_out/mlp4_time.log 2>&1 || exit 5
rm -f gpurun_out/prof_mlp4/run_kernel_trace.csv
echo done
