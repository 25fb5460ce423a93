# A/B of libppomlp builds: per-launch timing of one fused optimizer step for each, then the fused-PPO GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=unitree-rl-gym_amd/csrc/build
for v in ${AB_VARIANTS:-old}; do
  PPOMLP_LIB=$PWD/$B/libppomlp_$v.so timeout -k 10 120 python tools/probes/update_step_time.py > gpurun_out/ab_$v.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/probes/update_step_time.py > gpurun_out/ab_new.log 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_ppo.py tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit 3
echo done
