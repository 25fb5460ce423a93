# Profile set of the fused env step (rounds 5-6): per config a kernel trace, FETCH_SIZE / WRITE_SIZE
# passes (separate, each with a 1 GiB reference copy), two SQ instruction-mix passes and the
# per-phase stamps build; for Go2 also the traffic passes of the I/O-only diagnostic build
# (make -C unitree-rl-gym_amd/csrc iodiag: the step's global loads and stores without the
# physics), the known-byte calibration of the counters for this access pattern
# (tools/traffic_calib.py).
# usage: [PROF=gpurun_out/prof] bash tools/gpu_env_profile.sh [task:envs ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFGS="${@:-go2:4096 h1:8192 h1_2:8192 g1:4096}"
B=unitree-rl-gym_amd/csrc/build
for cfg in $CFGS; do
  task=${cfg%%:*}; n=${cfg##*:}
  O=${PROF:-gpurun_out/prof}/${task}_$n
  rm -rf $O && mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python tools/profile_env.py $task $n 60 > $O/trace.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python tools/profile_env.py $task $n 20 > $O/fetch.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python tools/profile_env.py $task $n 20 > $O/write.log 2>&1 || exit 4
  python tools/pmc_summary.py $O/trace $O/fetch $O/write "k_step<" $O/pmc_k_step.json > $O/pmc.log 2>&1 || exit 5
  if [ "$task" = "go2" ]; then
    export LEGGEDSIM_LIB=$B/libleggedsim_io.so
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/io_trace -o run --output-format csv -- python tools/profile_env.py $task $n 20 > $O/io_trace.log 2>&1 || exit 12
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/io_fetch -o run --output-format csv -- python tools/profile_env.py $task $n 20 > $O/io_fetch.log 2>&1 || exit 13
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/io_write -o run --output-format csv -- python tools/profile_env.py $task $n 20 > $O/io_write.log 2>&1 || exit 14
    unset LEGGEDSIM_LIB
    python tools/pmc_summary.py $O/io_trace $O/io_fetch $O/io_write "k_step<" $O/pmc_k_step_io_only.json > $O/pmc_io.log 2>&1 || exit 15
    python tools/traffic_calib.py $O/pmc_k_step.json $O/pmc_k_step_io_only.json $n $O/traffic_calib.json > $O/calib.log 2>&1 || exit 16
  fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/sq1 -o run --output-format csv -- python tools/profile_env.py $task $n 8 > $O/sq1.log 2>&1 || exit 6
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/sq2 -o run --output-format csv -- python tools/profile_env.py $task $n 8 > $O/sq2.log 2>&1 || exit 7
  python tools/sq_summary.py $O/sq1 $O/sq2 $O/sq_k_step.json > $O/sq.log 2>&1 || exit 8
  LEGGEDSIM_LIB=$B/libleggedsim_stamps.so timeout -k 10 200 python tools/phase_stamps.py $task $n > $O/phase_stamps.txt 2>&1 || exit 9
  find $O -name "*kernel_trace.csv" -delete; find $O -name "*counter_collection.csv" -size +2M -delete
  echo "$cfg done"
done
echo done
