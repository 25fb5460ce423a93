#!/bin/bash
# memory-path counters of the update's kernels (tools/probes/update_step_time.py), one pass per block set
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/upd_mem
rm -rf $O && mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL -d $O/p1 -o run --output-format csv -- python tools/probes/update_step_time.py > $O/p1.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD TCC_HIT TCC_MISS -d $O/p2 -o run --output-format csv -- python tools/probes/update_step_time.py > $O/p2.log 2>&1 || exit 3
python tools/pmc_mem_kernels.py $O/p1 $O/p2 > $O/summary.txt || exit 5
find $O -name "*counter_collection.csv" -size +4M -delete
cat $O/summary.txt
