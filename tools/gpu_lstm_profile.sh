#!/bin/bash
# SQ counters of the recurrent kernels over H1 x 8192 PPO iterations (tools/ppo_breakdown.py):
# two counter passes, summarised per kernel and grid size (tools/lstm_sq_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lstmprof
rm -rf $O && mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/sq1 -o run --output-format csv -- python tools/ppo_breakdown.py ${1:-h1} ${2:-8192} 1 > $O/sq1.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/sq2 -o run --output-format csv -- python tools/ppo_breakdown.py ${1:-h1} ${2:-8192} 1 > $O/sq2.log 2>&1 || exit 3
python tools/lstm_sq_summary.py $O/sq1 $O/sq2 $O/lstm_sq.json > $O/summary.txt 2>&1 || exit 4
find $O -name "*counter_collection.csv" -delete
cat $O/summary.txt
