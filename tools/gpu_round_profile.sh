# Round profile set: k_step kernel trace + FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md HBM
# recipe, separate passes), the default bench line, and a kernel trace of bench.py itself.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python tools/profile_env.py go2 4096 100 > gpurun_out/prof_trace.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > gpurun_out/prof_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > gpurun_out/prof_write.log 2>&1 || exit 4
python tools/pmc_summary.py gpurun_out/prof_trace gpurun_out/prof_fetch gpurun_out/prof_write k_step gpurun_out/pmc_k_step.json || exit 5
rm -f gpurun_out/prof_trace/run_kernel_trace.csv gpurun_out/prof_fetch/run_counter_collection.csv.gz gpurun_out/prof_write/run_counter_collection.csv.gz
rm -rf gpurun_out/prof_sq gpurun_out/prof_sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/prof_sq -o run --output-format csv -- python tools/profile_env.py go2 4096 10 > gpurun_out/prof_sq.log 2>&1 || exit 9
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/prof_sq2 -o run --output-format csv -- python tools/profile_env.py go2 4096 10 > gpurun_out/prof_sq2.log 2>&1 || exit 10
python tools/sq_summary.py gpurun_out/prof_sq gpurun_out/prof_sq2 gpurun_out/sq_k_step.json > /dev/null || exit 11
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 6
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no_cpu_baseline --no_other_configs > gpurun_out/prof_bench.log 2>&1 || exit 7
python tools/iter_trace.py gpurun_out/prof_bench/run_kernel_trace.csv > gpurun_out/iteration_breakdown.txt 2>&1 || exit 8
rm -f gpurun_out/prof_bench/run_kernel_trace.csv
cat gpurun_out/bench.json
echo done
