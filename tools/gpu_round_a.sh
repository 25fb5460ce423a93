set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python tools/profile_env.py go2 4096 100 > gpurun_out/prof_trace.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > gpurun_out/prof_fetch.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > gpurun_out/prof_write.log 2>&1 || exit 4
echo done
