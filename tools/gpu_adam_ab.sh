#!/bin/bash
# k_adam (PMLP_ADAM_VEC=1) against k_adam_vec<4> on the captured Go2 update: the update A/B
# with bitwise parameter comparisons (tools/gpu_update_ab.sh), the kernels' own durations from a
# rocprofv3 kernel trace of each, the fused-PPO and update-replay GPU tests.
# log: gpurun_out/adam/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/adam
rm -rf $O gpurun_out/update_ab.log gpurun_out/update_ab_full.log && mkdir -p $O
L=$PWD/unitree-rl-gym_amd/csrc/build/libppomlp.so
A_ENV='PMLP_ADAM_VEC=1' bash tools/gpu_update_ab.sh $L $L || exit 1
cp gpurun_out/update_ab.log $O/ab_vec1_vs_vec4.log
for v in 1 4; do
  PMLP_ADAM_VEC=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python tools/probes/update_time.py $O/p$v.npz > $O/prof_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_update_replay.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
cat $O/ab_*.log
python - <<'PY'
import sqlite3, statistics as S
for v in (1, 4):
    db = sqlite3.connect(f"gpurun_out/adam/prof_{v}/run_results.db")
    d = [r[0] for r in db.execute("select duration from kernels where name like '%k_adam%'")]
    print(f"PMLP_ADAM_VEC={v}: Adam kernel median {S.median(d) / 1e3:.2f} us over {len(d)} launches")
PY
tail -n 3 $O/tests.log
exit $rc
