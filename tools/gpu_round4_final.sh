# Round-4 closing measurements of the shipped build, one box: the post-physics prefetch A/B
# (build/libleggedsim_pre.so, not shipped), the full GPU suite, smoke, the default bench line
# and the Go2 profile set (tools/gpu_round4_profile.sh).  Every step under its own time limit;
# the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
B=unitree-rl-gym_amd/csrc/build
O=gpurun_out/final2
mkdir -p $O
TIME_KSTEP_ACTIONS=zero timeout -k 10 300 python tools/time_kstep.py go2 4096 $B/libleggedsim.so $B/libleggedsim_pre.so \
  $B/libleggedsim.so $B/libleggedsim_pre.so > $O/ab_pre.txt 2>&1 || exit 1
bash tools/gpu_tests.sh tests -m gpu; rc=$?; cp gpurun_out/tests.log $O/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 3
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 4
bash tools/gpu_round4_profile.sh go2:4096 || exit 5
echo final2 done
