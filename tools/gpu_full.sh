#!/bin/bash
# the round-end GPU checks: every -m gpu test, then smoke()
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; echo smoke=$rc; exit $rc
