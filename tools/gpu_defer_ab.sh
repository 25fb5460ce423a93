#!/bin/bash
# The env's extras in the rollout's launches (default) against the env's own extras launch
# (ROLL_DEFER=0): the captured Go2 4096 rollout's median replay, 3 interleaved rounds, the
# bitwise comparison of the rollout storage and parameters, then the bench under the kernel
# trace (tools/gpu_iter_profile.sh).  Log: gpurun_out/defer_ab/ab.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/defer_ab
rm -rf $O && mkdir -p $O
for rep in 1 2 3; do
  for d in 1 0; do
    ROLL_DEFER=$d timeout -k 10 240 python tools/probes/rollout_time.py $O/roll_${d}_$rep.json > $O/time_${d}_$rep.log 2>&1 || exit 1
    grep rollout $O/time_${d}_$rep.log >> $O/ab.log
  done
done
python - >> $O/ab.log 2>&1 <<'PY'
import json
a, b = (json.load(open(f"gpurun_out/defer_ab/roll_{d}_1.json")) for d in (1, 0))
bad = [k for k in a if a[k] != b[k]]
print("defer vs own launch: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
PY
bash tools/gpu_iter_profile.sh > $O/iter.log 2>&1 || exit 2
cp gpurun_out/iterprof/iteration_breakdown.txt $O/
cat $O/ab.log
head -12 $O/iteration_breakdown.txt
