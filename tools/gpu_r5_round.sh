#!/bin/bash
# one box: env-kernel parity + k_step A/B of the candidate builds, then the full GPU suite,
# smoke and the default bench line of the shipped build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=unitree-rl-gym_amd/csrc/build
LIBS="${LIBS:-$B/libleggedsim_base.so default}" bash tools/gpu_kstep_ab.sh || exit 2
OUT=${OUT:-r5d} bash tools/gpu_check.sh || exit 3
