#!/bin/bash
# The LSTM sequence kernels with their per-step inputs loaded two steps ahead (this build) against
# the previous build (libppomlp_prev.so, one step ahead): the H1 x 8192 update replay (ms), the
# H1 x 8192 and G1 x 4096 rollouts + two iterations (digests compared), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/lstm_prefetch2; rm -rf $O; mkdir -p $O
B=$PWD/unitree-rl-gym_amd/csrc/build
for L in libppomlp_prev.so libppomlp.so libppomlp_prev.so libppomlp.so; do
  PPOMLP_LIB=$B/$L timeout -k 10 300 python tools/probes/update_race.py 300 > $O/upd.log 2>&1 || exit 1
  echo "$L $(grep 'update replays' $O/upd.log)" >> $O/ab.log
done
for task in "h1 8192" "g1 4096"; do
  set -- $task
  for L in libppomlp_prev.so libppomlp.so; do
    PPOMLP_LIB=$B/$L ROLL_TASK=$1 ROLL_ENVS=$2 timeout -k 10 300 python tools/probes/rollout_time.py $O/roll_$1_$L.json > $O/t.log 2>&1 || exit 1
    grep rollout $O/t.log >> $O/ab.log
  done
  python - $1 >> $O/ab.log 2>&1 <<'PY'
import json, sys
t = sys.argv[1]
a, b = (json.load(open(f"gpurun_out/lstm_prefetch2/roll_{t}_{L}.json")) for L in ("libppomlp_prev.so", "libppomlp.so"))
bad = [k for k in a if a[k] != b[k]]
print(f"{t}: two steps ahead vs one: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
PY
done
cat $O/ab.log
