#!/bin/bash
# A/B of libppomlp.so builds on the captured Go2 rollout (tools/probes/rollout_time.py),
# interleaved in separate processes (A B C.. A B C..), plus bitwise comparisons of the
# rollout storage and parameters after two seeded iterations: each build against itself and
# against the first.
# usage: tools/gpu_rollout_ab.sh libA.so libB.so [libC.so ...]   (log: gpurun_out/rollout_ab.log)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rm -f gpurun_out/rollout_ab.log gpurun_out/rollout_ab_full.log
for rep in 1 2 3; do
  i=0
  for lib in "$@"; do
    PPOMLP_LIB=$lib timeout -k 10 240 python tools/probes/rollout_time.py gpurun_out/roll_${i}_$rep.json >> gpurun_out/rollout_ab_full.log 2>&1 || exit 1
    i=$((i + 1))
  done
done
python - $# >> gpurun_out/rollout_ab.log 2>&1 <<'PY'
import json, sys
def cmp(x, y):
    a, b = (json.load(open(f"gpurun_out/roll_{z}.json")) for z in (x, y))
    bad = [k for k in a if a[k] != b[k]]
    print(f"{x} vs {y}: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:6]}"))
for i in range(int(sys.argv[1])):
    cmp(f"{i}_1", f"{i}_2")
    if i:
        cmp("0_1", f"{i}_1")
PY
grep "rollout .* ms median" gpurun_out/rollout_ab_full.log >> gpurun_out/rollout_ab.log
cat gpurun_out/rollout_ab.log
