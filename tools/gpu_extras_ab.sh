# k_step_extras with batched loads (build/libleggedsim_ex.so) vs the shipped build: parity/env/plugin/script GPU tests on the new build, kernel-trace stats of a 60-step Go2 4096 run per build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=$PWD/unitree-rl-gym_amd/csrc/build
O=gpurun_out/ab_ex
mkdir -p $O
LEGGEDSIM_LIB=$B/libleggedsim_ex.so bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_env.py tests/test_gpu_plugin.py tests/test_gpu_scripts.py -x || exit 1
cp gpurun_out/tests.log $O/tests.txt
for lib in libleggedsim.so libleggedsim_ex.so; do
  LEGGEDSIM_LIB=$B/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${lib%.so} -o run --output-format csv -- python tools/profile_env.py go2 4096 60 > $O/${lib%.so}.log 2>&1 || exit 2
done
find $O -name "*kernel_trace.csv" -delete
for lib in libleggedsim libleggedsim_ex; do echo "$lib: $(grep -h k_step_extras $O/$lib/run_kernel_stats.csv | cut -c1-200)"; done
tail -1 $O/tests.txt
