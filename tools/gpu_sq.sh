# SQ issue/stall counters of the env kernel (one pass, SQ block only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_sq gpurun_out/prof_sq2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/prof_sq -o run --output-format csv -- python tools/profile_env.py go2 4096 10 > gpurun_out/prof_sq.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/prof_sq2 -o run --output-format csv -- python tools/profile_env.py go2 4096 10 > gpurun_out/prof_sq2.log 2>&1 || exit 3
echo done
