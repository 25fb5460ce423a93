#!/bin/bash
# GEMM time split: the shipped library against diagnostic builds without the result stores
# and without the k-loop operand loads (make -C unitree-rl-gym_amd/csrc diag)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B=unitree-rl-gym_amd/csrc/build
run() { echo "== $*"; env "$@" timeout -k 10 200 python tools/probes/update_step_time.py | grep -E "PART_TN|BWD_DX|FWD|reduce|TOTAL" || exit 3; }
run PPOMLP_LIB=$B/libppomlp.so
run PPOMLP_LIB=$B/libppomlp_nostore.so
run PPOMLP_LIB=$B/libppomlp_noload.so
