#!/bin/bash
# wave timelines and phase stamps of the fused env step, stamps build
# (needs libleggedsim_stamps.so un-ignored in .gpurunignore for the call)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export LEGGEDSIM_LIB=unitree-rl-gym_amd/csrc/build/libleggedsim_stamps.so
for cfg in ${@:-go2:4096 h1:8192 h1_2:8192 g1:4096}; do
  task=${cfg%%:*}; n=${cfg##*:}
  O=${PROF:-gpurun_out/prof}/${task}_$n
  mkdir -p $O
  timeout -k 10 120 python tools/wave_timeline.py $task $n 0.5 > $O/wave_timeline.txt 2>&1 || exit 2
  timeout -k 10 120 python tools/phase_stamps.py $task $n > $O/phase_stamps.txt 2>&1 || exit 3
  echo "$cfg done"
done
