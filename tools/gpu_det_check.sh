#!/bin/bash
# Run-to-run determinism of recurrent training (H1 x 8192, two seeded iterations: eager, then
# captured): the rollout probe 3 times per configuration, digests compared (gpurun_out/det/).
# usage: tools/gpu_det_check.sh "ENV=VAL ..." "ENV=VAL ..." ...   (one configuration per argument)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/det
rm -rf $O && mkdir -p $O
i=0
for cfg in "$@"; do
  for rep in 1 2 3; do
    env $cfg ROLL_TASK=${TASK:-h1} ROLL_ENVS=${ENVS:-8192} timeout -k 10 300 python tools/probes/rollout_time.py $O/r_${i}_$rep.json > $O/t_${i}_$rep.log 2>&1 || exit 1
  done
  echo "$i: $cfg" >> $O/configs.txt
  i=$((i + 1))
done
python - $i >> $O/summary.txt 2>&1 <<'PY'
import itertools, json, sys
n = int(sys.argv[1])
d = {(c, r): json.load(open(f"gpurun_out/det/r_{c}_{r}.json")) for c in range(n) for r in (1, 2, 3)}
for a, b in itertools.combinations(sorted(d), 2):
    bad = [k for k in d[a] if d[a][k] != d[b][k]]
    print(a, b, "equal" if not bad else f"{len(bad)} differ: {bad[:8]}")
PY
cat $O/configs.txt $O/summary.txt
