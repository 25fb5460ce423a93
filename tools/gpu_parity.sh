#!/bin/bash
# GPU parity suite (bitwise HIP == oracle); logs under gpurun_out/.  Extra args go to pytest.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/parity.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E  .*differ|passed|failed" gpurun_out/parity.log | tail -40
exit $rc
