#!/bin/bash
# per-launch update-step timing under the GEMM tile / split-K knobs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
run() { echo "== $*"; env "$@" timeout -k 10 200 python tools/probes/update_step_time.py | grep -E "PART_TN|BWD_DX|FWD|reduce|TOTAL" || exit 3; }
run PMLP_WIDE_TILE=0
run PMLP_WIDE_TILE=1
run PMLP_WIDE_TILE=1 PMLP_KSPLIT_TARGET=128
run PMLP_WIDE_TILE=1 PMLP_KSPLIT_TARGET=64
run PMLP_WIDE_TILE=0 PMLP_KSPLIT_TARGET=128
