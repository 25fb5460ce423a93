# bench + phase stamps + kernel trace of full PPO iterations (bench.py itself)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
LEGGEDSIM_LIB=$PWD/unitree-rl-gym_amd/csrc/build/libleggedsim_stamps.so timeout -k 10 200 python tools/phase_stamps.py go2 4096 > gpurun_out/stamps.log 2>&1 || exit 2
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no_cpu_baseline > gpurun_out/prof_bench.log 2>&1 || exit 3
echo done
