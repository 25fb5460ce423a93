#!/bin/bash
# Forward-GEMM load-ring depth (PMLP_PF_FWD) on the whole PPO iteration: the rollout's
# 4096-row forward GEMMs (small grids, latency-bound k-loops) and the update's forwards;
# two interleaved rounds of bench.py, Go2 4096
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pf_ab
mkdir -p $O
for r in 1 2; do
  for pf in 1 2 3; do
    PMLP_PF_FWD=$pf timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no_cpu_baseline --no_other_configs \
        > $O/pf${pf}_r$r.json 2> $O/pf${pf}_r$r.err || exit 3
    tail -1 $O/pf${pf}_r$r.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('PMLP_PF_FWD=$pf round $r', 'ms/iter', d['ms_per_step'], 'rollout', round(d['rollout_env_steps_per_s']/1e6, 3), 'M/s')"
  done
done
