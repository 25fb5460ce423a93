# PPO GPU tests + default bench (no other-config legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ppo_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --no_other_configs > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['env_step_kernel_ms'])"
echo done
