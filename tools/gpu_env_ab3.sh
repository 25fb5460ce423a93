# three-way A/B of libleggedsim builds (old / current / variant), k_step time, then env parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/unitree-rl-gym_amd/csrc/build
V=${VARIANT:-nb}
timeout -k 10 400 python tools/time_kstep.py ${TASK:-go2} ${NENV:-4096} $B/libleggedsim_old.so $B/libleggedsim.so $B/libleggedsim_$V.so $B/libleggedsim_old.so $B/libleggedsim.so $B/libleggedsim_$V.so > gpurun_out/env_ab3.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py -x -q --timeout 120 --timeout-method thread > gpurun_out/env_tests.log 2>&1 || exit 2
grep "k_step median" gpurun_out/env_ab3.log
tail -1 gpurun_out/env_tests.log
