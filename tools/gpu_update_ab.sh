#!/bin/bash
# A/B of two libppomlp.so builds on the captured Go2 PPO update, interleaved in separate
# processes (A B A B), plus a bitwise comparison of the parameters both give after 3 updates.
# usage: tools/gpu_update_ab.sh libA.so libB.so   (log: gpurun_out/update_ab.log)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$1; B=$2
for rep in 1 2; do
  PPOMLP_LIB=$A timeout -k 10 240 python tools/probes/update_time.py gpurun_out/upd_a.npz >> gpurun_out/update_ab.log 2>&1 || exit 1
  PPOMLP_LIB=$B timeout -k 10 240 python tools/probes/update_time.py gpurun_out/upd_b.npz >> gpurun_out/update_ab.log 2>&1 || exit 1
done
python - >> gpurun_out/update_ab.log 2>&1 <<'PY'
import numpy as np
a, b = np.load("gpurun_out/upd_a.npz"), np.load("gpurun_out/upd_b.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print("params bitwise equal" if not bad else f"params differ: {bad}")
PY
cat gpurun_out/update_ab.log
