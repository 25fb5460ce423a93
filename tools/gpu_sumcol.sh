#!/bin/bash
# the PARTIAL_TN bias column as a ones product: parity tests, then the optimizer-step timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_ppo.py 2>&1 | tail -4 || exit 2
timeout -k 10 200 python tools/probes/update_step_time.py | grep -E "PART_TN|BWD_DX|FWD|reduce|TOTAL" || exit 3
