#!/bin/bash
# A/B of libleggedsim.so builds on the captured Go2 rollout: per build, the kernel trace of
# tools/probes/rollout_time.py (per-kernel averages from rocprofv3 --stats) and, interleaved
# over 3 rounds, the rollout's median replay time; plus the bitwise comparison of the rollout
# storage and parameters after two seeded iterations (each build against the first).
# usage: tools/gpu_lgs_ab.sh libA.so libB.so [...]   (log: gpurun_out/lgs_ab/ab.log)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/lgs_ab
rm -rf $O && mkdir -p $O
i=0
for lib in "$@"; do
  LEGGEDSIM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$i -o run --output-format csv -- python tools/probes/rollout_time.py $O/roll_${i}_0.json > $O/prof_$i.log 2>&1 || exit 1
  python tools/kernel_stats_top.py $O/prof_$i 8 > $O/stats_$i.txt 2>&1
  find $O/prof_$i -name "*kernel_trace.csv" -delete
  echo "== $lib" >> $O/ab.log; head -8 $O/stats_$i.txt >> $O/ab.log
  i=$((i + 1))
done
for rep in 1 2 3; do
  i=0
  for lib in "$@"; do
    LEGGEDSIM_LIB=$lib timeout -k 10 240 python tools/probes/rollout_time.py $O/roll_${i}_$rep.json > $O/time_${i}_$rep.log 2>&1 || exit 2
    echo "$(basename $lib) rep $rep: $(grep 'rollout' $O/time_${i}_$rep.log)" >> $O/ab.log
    i=$((i + 1))
  done
done
python - $# >> $O/ab.log 2>&1 <<'PY'
import json, sys
for i in range(1, int(sys.argv[1])):
    a, b = (json.load(open(f"gpurun_out/lgs_ab/roll_{z}_1.json")) for z in (0, i))
    bad = [k for k in a if a[k] != b[k]]
    print(f"build {i} vs 0: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
PY
cat $O/ab.log
