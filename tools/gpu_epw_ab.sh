#!/bin/bash
# A/B of the Go2 env-step kernel: one env per wave vs two (LGS_ENVS_PER_WAVE), interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  LGS_ENVS_PER_WAVE=1 timeout -k 10 120 python tools/time_kstep.py go2 4096 || exit 3
  timeout -k 10 120 python tools/time_kstep.py go2 4096 || exit 4
done
