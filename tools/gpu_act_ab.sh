# k_act4 vs k_act: rollout-path kernel times in a bench trace for both libraries, then PPO + env tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/unitree-rl-gym_amd/csrc/build
for v in old new old new; do
  L=$B/libppomlp.so; [ $v = old ] && L=$B/libppomlp_old.so
  PPOMLP_LIB=$L timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no_cpu_baseline --no_other_configs > gpurun_out/act_$v.json 2>/dev/null || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/act_$v.json'));print(d['value'],d['ms_per_step'],d['rollout_env_steps_per_s'])")"
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > gpurun_out/act_tests.log 2>&1 || exit 2
tail -1 gpurun_out/act_tests.log
