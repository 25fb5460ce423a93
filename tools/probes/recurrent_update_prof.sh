# Recurrent update at H1 scale: wall times (eager / captured) and a kernel trace of two eager
# updates summarised as per-kernel totals per optimizer step (40 steps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/rec_upd
rm -rf $O && mkdir -p $O
timeout -k 10 200 python tools/probes/recurrent_update_time.py > $O/time.txt 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python tools/probes/recurrent_update_time.py --trace > $O/tr.log 2>&1 || exit 3
python tools/kernel_stats_top.py $O/tr 40 > $O/top.txt 2>&1 || exit 4
find $O -name "*kernel_trace.csv" -delete
cat $O/time.txt $O/top.txt
