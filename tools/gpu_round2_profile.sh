# Round-2 profile set of the Go2 4096-env step kernel: kernel trace, calibrated
# FETCH_SIZE / WRITE_SIZE passes (separate; each with a 1 GiB reference copy),
# two SQ instruction-mix passes, then a kernel trace of bench.py itself.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2prof
rm -rf $O && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python tools/profile_env.py go2 4096 100 > $O/trace.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > $O/fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python tools/profile_env.py go2 4096 30 > $O/write.log 2>&1 || exit 4
python tools/pmc_summary.py $O/trace $O/fetch $O/write "k_step<" $O/pmc_k_step.json || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/sq1 -o run --output-format csv -- python tools/profile_env.py go2 4096 10 > $O/sq1.log 2>&1 || exit 9
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/sq2 -o run --output-format csv -- python tools/profile_env.py go2 4096 10 > $O/sq2.log 2>&1 || exit 10
python tools/sq_summary.py $O/sq1 $O/sq2 $O/sq_k_step.json > /dev/null || exit 11
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no_cpu_baseline --no_other_configs > $O/bench.log 2>&1 || exit 7
python tools/iter_trace.py $O/bench/run_kernel_trace.csv > $O/iteration_breakdown.txt 2>&1 || exit 8
find $O -name "*kernel_trace.csv" -delete; find $O -name "*counter_collection.csv" -size +2M -delete
cat $O/pmc_k_step.json
echo done
