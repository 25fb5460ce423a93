#!/bin/bash
# The recurrent heads kernels on the update's shape (tools/probes/heads_time.py): median times
# per build named on the command line (default: the shipped libppomlp.so), then, for the first
# build, the SQ instruction mix and wave-time shares of k_heads_fwd / k_heads_bwd (two counter
# passes) and FETCH / WRITE.  Log: gpurun_out/heads/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/heads
rm -rf $O && mkdir -p $O
LIBS=${@:-unitree-rl-gym_amd/csrc/build/libppomlp.so}
for rep in 1 2; do
  for lib in $LIBS; do
    PPOMLP_LIB=$lib timeout -k 10 120 python tools/probes/heads_time.py >> $O/times.txt 2>&1 || exit 1
  done
done
first=$(echo $LIBS | cut -d' ' -f1)
export PPOMLP_LIB=$first
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/sq1 -o run --output-format csv -- python tools/probes/heads_time.py > $O/sq1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/sq2 -o run --output-format csv -- python tools/probes/heads_time.py > $O/sq2.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python tools/probes/heads_time.py > $O/fetch.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python tools/probes/heads_time.py > $O/write.log 2>&1 || exit 5
for k in "k_heads_fwd<" "k_heads_bwd<"; do
  python tools/sq_summary.py $O/sq1 $O/sq2 $O/sq_$(echo $k | tr -d '<').json "$k" > /dev/null 2>&1
done
find $O -name "*.csv" -size +2M -delete
cat $O/times.txt
