#!/bin/bash
# A/B of the GEMM load-ring depth (PMLP_PF_TN / _DX / _FWD) on one optimizer step, then
# the fused-PPO parity tests with every ring at depth 3
cd "${GRAFT_REPO_ROOT:-/root/repo}"
run() { echo "== $*"; env "$@" timeout -k 10 200 python tools/probes/update_step_time.py | grep -E "PART_TN|BWD_DX|FWD|reduce|TOTAL" || exit 3; }
run PMLP_PF_TN=1
run PMLP_PF_TN=2
run PMLP_PF_TN=3
run PMLP_PF_DX=2
run PMLP_PF_DX=3
run PMLP_PF_FWD=2
run PMLP_PF_FWD=3
run PMLP_PF_TN=3 PMLP_PF_DX=3 PMLP_PF_FWD=3 PMLP_KSPLIT_TARGET=64
PMLP_PF_TN=3 PMLP_PF_DX=3 PMLP_PF_FWD=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_ppo.py 2>&1 | tail -3
