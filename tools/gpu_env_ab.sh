# A/B of libleggedsim builds (k_step time, HIP events) + the env GPU parity tests on the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/unitree-rl-gym_amd/csrc/build
timeout -k 10 400 python tools/time_kstep.py ${TASK:-go2} ${NENV:-4096} $B/libleggedsim_old.so $B/libleggedsim.so $B/libleggedsim_old.so $B/libleggedsim.so $B/libleggedsim_old.so $B/libleggedsim.so > gpurun_out/env_ab.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > gpurun_out/env_tests.log 2>&1 || exit 2

echo done
