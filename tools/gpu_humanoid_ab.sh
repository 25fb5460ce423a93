#!/bin/bash
# humanoid step kernel: bitwise parity vs the oracle, then A/B of the previous build vs this
# one (and any extra variant builds present)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=unitree-rl-gym_amd/csrc/build
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_self_collision.py > gpurun_out/hum_parity.log 2>&1
rc=$?; tail -3 gpurun_out/hum_parity.log; [ $rc -eq 0 ] || exit 2
LIBS="$PWD/$B/libleggedsim_prev.so $PWD/$B/libleggedsim.so"
[ -f $B/libleggedsim_w3.so ] && LIBS="$LIBS $PWD/$B/libleggedsim_w3.so"
for t in "h1 8192" "g1 4096" "h1_2 8192" "go2 4096"; do
  timeout -k 10 300 python tools/time_kstep.py $t $LIBS || exit 3
done
