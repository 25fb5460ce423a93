#!/bin/bash
# round-5 profile set, part A: Go2 4096 and H1_2 8192 env kernels, the Go2 iteration breakdown
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_round5_profile.sh go2:4096 h1_2:8192 || exit 2
bash tools/gpu_iter_profile.sh || exit 3
