#!/bin/bash
# env-kernel change: the bit-exact parity suite (SKIP_TESTS=1: none), then k_step of each build
# in LIBS (paths, "default" = the shipped build/libleggedsim.so), alternating, per BASELINE config
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/kstep_ab
mkdir -p $O
[ -n "$SKIP_TESTS" ] || { bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_gpu_contact_slots.py tests/test_gpu_self_collision.py \
    tests/test_gpu_padded.py tests/test_gpu_plugin.py -x; rc=$?; cp gpurun_out/tests.log $O/tests.txt; [ $rc -eq 0 ] || exit 2; }
B=unitree-rl-gym_amd/csrc/build
LIBS=${LIBS:-"$B/libleggedsim_base.so default"}
: > $O/kstep.txt
for cfg in "go2 4096" "g1_rough 4096" "h1 8192" "h1_2 8192"; do
  for rep in 1 2; do
    for lib in $LIBS; do
      if [ "$lib" = default ]; then l=""; else l=$lib; fi
      echo -n "$(basename ${lib}) " >> $O/kstep.txt
      LEGGEDSIM_LIB=$l timeout -k 10 120 python tools/time_kstep.py $cfg 2>&1 | grep k_step >> $O/kstep.txt || exit 3
    done
  done
done
cat $O/kstep.txt
