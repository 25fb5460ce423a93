#!/bin/bash
# A/B of two libppomlp.so builds on the captured Go2 PPO update, interleaved in separate
# processes (A B A B), plus bitwise comparisons of the parameters after 3 updates: A vs A and
# B vs B (run-to-run determinism), A vs B.
# usage: [A_ENV='VAR=value ...'] tools/gpu_update_ab.sh libA.so libB.so   (log: gpurun_out/update_ab.log)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$1; B=$2
for rep in 1 2; do
  env $A_ENV PPOMLP_LIB=$A timeout -k 10 240 python tools/probes/update_time.py gpurun_out/upd_a$rep.npz >> gpurun_out/update_ab_full.log 2>&1 || exit 1
  PPOMLP_LIB=$B timeout -k 10 240 python tools/probes/update_time.py gpurun_out/upd_b$rep.npz >> gpurun_out/update_ab_full.log 2>&1 || exit 1
done
python - >> gpurun_out/update_ab.log 2>&1 <<'PY'
import numpy as np
def cmp(x, y):
    a, b = np.load(f"gpurun_out/upd_{x}.npz"), np.load(f"gpurun_out/upd_{y}.npz")
    d = max(float(np.abs(a[k].astype(np.float64) - b[k]).max()) for k in a.files)
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print(f"{x} vs {y}: " + ("bitwise equal" if not bad else f"{len(bad)} tensors differ, max |d| {d:.3e}"))
cmp("a1", "a2"); cmp("b1", "b2"); cmp("a1", "b1")
PY
grep "update .* ms median" gpurun_out/update_ab_full.log >> gpurun_out/update_ab.log
cat gpurun_out/update_ab.log
