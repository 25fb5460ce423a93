#!/bin/bash
# optimizer-step timing under the tile / split-K knobs (current kernels)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
run() { echo "== $*"; env "$@" timeout -k 10 200 python tools/probes/update_step_time.py | grep -E "PART_TN|BWD_DX|FWD|reduce|TOTAL" || exit 3; }
run PMLP_BIG_TILE=-1
run PMLP_BIG_TILE=0
run PMLP_BIG_TILE=2
run PMLP_KSPLIT_TARGET=256
run PMLP_KSPLIT_TARGET=64
