#!/bin/bash
# Run GPU test files (args) one pytest process; log under gpurun_out/tests.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest "$@" -v --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|^E  |passed|failed" gpurun_out/tests.log | tail -60
exit $rc
