# k_step A/B (previous vs current libleggedsim, alternating) + all GPU tests + default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/unitree-rl-gym_amd/csrc/build
timeout -k 10 400 python tools/time_kstep.py go2 4096 $B/libleggedsim_old.so $B/libleggedsim.so $B/libleggedsim_old.so $B/libleggedsim.so > gpurun_out/env_ab.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --no_other_configs > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3
cat gpurun_out/bench.json
echo done
