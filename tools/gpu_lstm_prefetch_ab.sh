#!/bin/bash
# The LSTM step with the next env tile's inputs prefetched (this build) against the previous build
# (libppomlp_prev.so): captured H1 x 8192 and G1 x 4096 rollouts, interleaved, digests compared;
# then the env-tile sweep of this build (tools/gpu_lstm_tiles_ab.sh: every count bitwise the 1-tile run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/lstm_prefetch; rm -rf $O; mkdir -p $O
B=$PWD/unitree-rl-gym_amd/csrc/build
for task in "h1 8192" "g1 4096"; do
  set -- $task
  for rep in 1 2; do for L in libppomlp_prev.so libppomlp.so; do
    PPOMLP_LIB=$B/$L ROLL_TASK=$1 ROLL_ENVS=$2 timeout -k 10 300 python tools/probes/rollout_time.py $O/roll_$1_${L}_$rep.json > $O/t.log 2>&1 || exit 1
    grep rollout $O/t.log >> $O/ab.log
  done; done
  python - $1 >> $O/ab.log 2>&1 <<'PY'
import json, sys
t = sys.argv[1]
a, b = (json.load(open(f"gpurun_out/lstm_prefetch/roll_{t}_{L}_1.json")) for L in ("libppomlp_prev.so", "libppomlp.so"))
bad = [k for k in a if a[k] != b[k]]
print(f"{t}: prefetch vs previous: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
PY
done
bash tools/gpu_lstm_tiles_ab.sh > /dev/null || exit 1
cat gpurun_out/lstm_tiles/ab.log >> $O/ab.log
cat $O/ab.log
