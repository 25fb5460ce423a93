# default bench line + kernel trace of bench.py (per-iteration breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
rm -rf gpurun_out/prof_bench
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no_cpu_baseline > gpurun_out/prof_bench.log 2>&1 || exit 3
python tools/iter_trace.py gpurun_out/prof_bench/run_kernel_trace.csv > gpurun_out/iteration_breakdown.txt 2>&1 || exit 4
rm -f gpurun_out/prof_bench/run_kernel_trace.csv.gz; gzip gpurun_out/prof_bench/run_kernel_trace.csv
echo done
