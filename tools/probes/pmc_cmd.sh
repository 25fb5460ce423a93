# SQ counters (two passes) + kernel trace of any python workload, summarised per kernel
# (tools/pmc_kernels.py).  usage: bash tools/probes/pmc_cmd.sh OUTDIR python-args...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$1; shift
rm -rf $O && mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS -d $O/p1 -o run --output-format csv -- python "$@" > $O/p1.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM -d $O/p2 -o run --output-format csv -- python "$@" > $O/p2.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python "$@" > $O/tr.log 2>&1 || exit 4
python tools/pmc_kernels.py $O/p1 $O/p2 $O/tr > $O/summary.txt || exit 5
find $O -name "*counter_collection.csv" -size +4M -delete; find $O -name "*kernel_trace.csv" -delete
cat $O/summary.txt
