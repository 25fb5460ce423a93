#!/bin/bash
# The recurrent rollout with pmlp_act in the heads' launch (default) against the two launches
# (PMLP_HEADS_ACT=0): the captured H1 x 8192 and G1 x 4096 rollouts' median replays, 2
# interleaved rounds each, and the rollout storage + parameters compared bitwise.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/heads_act
rm -rf $O && mkdir -p $O
for task in "h1 8192" "g1 4096"; do
  set -- $task
  for rep in 1 2; do
    for f in 1 0; do
      ROLL_TASK=$1 ROLL_ENVS=$2 PMLP_HEADS_ACT=$f timeout -k 10 300 python tools/probes/rollout_time.py $O/roll_$1_${f}_$rep.json > $O/time_$1_${f}_$rep.log 2>&1 || exit 1
      echo "heads_act=$f $(grep rollout $O/time_$1_${f}_$rep.log)" >> $O/ab.log
    done
  done
  python - $1 >> $O/ab.log 2>&1 <<'PY'
import json, sys
t = sys.argv[1]
a, b = (json.load(open(f"gpurun_out/heads_act/roll_{t}_{f}_1.json")) for f in (1, 0))
bad = [k for k in a if a[k] != b[k]]
print(f"{t}: fused vs two launches: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
PY
done
cat $O/ab.log
