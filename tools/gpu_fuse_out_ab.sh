#!/bin/bash
# the output layer in the last hidden layer's epilogue: tests, then step / bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_ppo.py tests/test_gpu_env.py -k "fused or rollout" > gpurun_out/fo_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fo_tests.log; [ $rc -eq 0 ] || exit 2
for v in 0 1 0 1; do
  echo "== PMLP_FUSE_OUT=$v"; PMLP_FUSE_OUT=$v timeout -k 10 200 python tools/probes/update_step_time.py | grep -E "TOTAL" || exit 3
done
for v in 0 1; do
  echo "== bench PMLP_FUSE_OUT=$v"; PMLP_FUSE_OUT=$v timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no_cpu_baseline --no_other_configs 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['rollout_env_steps_per_s'])" || exit 4
done
