set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/unitree-rl-gym_amd/csrc/build
for t in g1 h1; do
timeout -k 10 300 python tools/time_kstep.py $t 4096 $B/libleggedsim_old.so $B/libleggedsim.so $B/libleggedsim_old.so $B/libleggedsim.so > gpurun_out/env_ab_$t.log 2>&1 || exit 1
done
grep "k_step median" gpurun_out/env_ab_*.log
