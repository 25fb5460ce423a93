#!/bin/bash
# The recurrent heads on the matrix cores (default) against the VALU form (PMLP_HEADS_MFMA=0):
# the heads probe at the update's and the rollout's rows (times + output digests, interleaved),
# the H1 x 8192 captured rollout + two iterations (storage / parameter digests), the H1 update's
# replay time, the recurrent GPU tests.  log: gpurun_out/heads_mfma/ab.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/heads_mfma
rm -rf $O && mkdir -p $O
for m in 49152 8192; do
  for rep in 1 2; do
    for f in 0 1; do
      PMLP_HEADS_MFMA=$f timeout -k 10 120 python tools/probes/heads_time.py $m > $O/heads_${m}_${f}_$rep.log 2>&1 || exit 1
      echo "mfma=$f $(grep 'heads fwd' $O/heads_${m}_${f}_$rep.log)" >> $O/ab.log
    done
  done
done
for f in 0 1; do
  ROLL_TASK=h1 ROLL_ENVS=8192 PMLP_HEADS_MFMA=$f timeout -k 10 300 python tools/probes/rollout_time.py $O/roll_$f.json > $O/roll_$f.log 2>&1 || exit 1
  echo "mfma=$f $(grep rollout $O/roll_$f.log)" >> $O/ab.log
done
python - >> $O/ab.log 2>&1 <<'PY'
import json
a, b = (json.load(open(f"gpurun_out/heads_mfma/roll_{f}.json")) for f in (0, 1))
bad = [k for k in a if a[k] != b[k]]
print("h1 x 8192, 2 iterations, VALU vs MFMA heads: " + ("bitwise equal" if not bad else f"{len(bad)} arrays differ: {bad[:8]}"))
PY
for f in 0 1 0 1; do  # the captured H1 x 8192 update replayed from one state: ms per replay
  PMLP_HEADS_MFMA=$f timeout -k 10 300 python tools/probes/update_race.py 300 > $O/upd_$f.log 2>&1 || exit 1
  echo "mfma=$f $(grep 'update replays' $O/upd_$f.log)" >> $O/ab.log
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_recurrent.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
cat $O/ab.log
tail -n 2 $O/tests.log
exit $rc
