#!/bin/bash
# The recurrent rollout's LSTM step at 1 / 2 / 4 / 8 env tiles per workgroup
# (PMLP_LSTM_STEP_TILES): the captured H1 x 8192 rollout's median replay, 2 interleaved rounds,
# and the rollout storage + parameters after two seeded iterations compared bitwise with the
# 1-tile run.  Log: gpurun_out/lstm_tiles/ab.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/lstm_tiles
rm -rf $O && mkdir -p $O
for rep in 1 2; do
  for t in 1 2 4 8; do
    ROLL_TASK=h1 ROLL_ENVS=8192 PMLP_LSTM_STEP_TILES=$t timeout -k 10 300 python tools/probes/rollout_time.py $O/roll_${t}_$rep.json > $O/time_${t}_$rep.log 2>&1 || exit 1
    grep rollout $O/time_${t}_$rep.log >> $O/ab.log
  done
done
python - >> $O/ab.log 2>&1 <<'PY'
import json
a = json.load(open("gpurun_out/lstm_tiles/roll_1_1.json"))
for t in (2, 4, 8):
    b = json.load(open(f"gpurun_out/lstm_tiles/roll_{t}_1.json"))
    bad = [k for k in a if a[k] != b[k]]
    print(f"{t} tiles vs 1: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
PY
cat $O/ab.log
