#!/bin/bash
# Round-6 profile set on one box (needs libleggedsim_stamps.so / libleggedsim_io.so un-ignored in
# .gpurunignore for the call): the Go2 4096 and H1_2 8192 env kernels (trace, calibrated
# FETCH/WRITE, SQ, phase stamps), the Go2 wave timeline, the bench iteration breakdown, and two
# more seeds of the Go2 300-iteration learning curve at 5 and 8 sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PROF=gpurun_out/prof6
bash tools/gpu_env_profile.sh go2:4096 h1_2:8192 || exit 2
bash tools/gpu_wave_timeline.sh go2:4096 || exit 3
bash tools/gpu_iter_profile.sh > /dev/null || exit 4
mkdir -p $PROF/learning
for seed in 2 3; do
  for sw in 5 8; do
    timeout -k 10 200 python tools/learn_curve.py go2 300 4096 - $sw $seed > $PROF/learning/go2_${sw}_sweeps_seed$seed.log 2>&1 || exit 5
  done
done
for f in $PROF/learning/*.log; do echo $f; tail -n 1 $f; done
