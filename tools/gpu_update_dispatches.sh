#!/bin/bash
# per-dispatch time and traffic counters of one captured fused optimizer step (Go2 update)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/upd_disp
rm -rf $O && mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python tools/probes/update_pair_ab.py > $O/trace.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python tools/probes/update_pair_ab.py > $O/fetch.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python tools/probes/update_pair_ab.py > $O/write.log 2>&1 || exit 4
python tools/probes/update_dispatches.py $O/trace $O/fetch $O/write > $O/table.txt 2>&1 || exit 5
find $O -name "*.csv" -size +2M -delete
cat $O/table.txt
