#!/bin/bash
# A/B of the fused env-step kernel on one box: every (task, envs) pair with each library given,
# interleaved (build A, build B, build A, ...) so box drift hits both.  Log: gpurun_out/kstep_ab.log
# usage: tools/gpu_ab_kstep.sh libA.so libB.so [task:n ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$1; B=$2; shift 2
PAIRS=${@:-go2:4096 h1:8192 h1_2:8192 g1:4096}
for rep in 1 2; do
  for p in $PAIRS; do
    t=${p%%:*}; n=${p##*:}
    for lib in $A $B; do
      timeout -k 10 240 python tools/time_kstep.py $t $n $lib >> gpurun_out/kstep_ab.log 2>&1 || exit 1
    done
  done
done
grep "k_step median" gpurun_out/kstep_ab.log
