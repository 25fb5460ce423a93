#!/bin/bash
# round-5 profile set, part B: H1 8192 and G1 4096 env kernels, the Go2 traffic-vs-envs sweep,
# the G1 contact-capacity A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_round5_profile.sh h1:8192 g1:4096 || exit 2
bash tools/gpu_traffic_sweep.sh || exit 3
mkdir -p gpurun_out/g1cap
timeout -k 10 400 python tools/g1_capacity_ab.py 300 > gpurun_out/g1cap/ab.txt 2>&1 || exit 4
