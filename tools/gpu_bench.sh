#!/bin/bash
# bench.py on the GPU box (N=1): JSON line -> gpurun_out/bench.json, stderr -> gpurun_out/bench.err
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -c 3000 gpurun_out/bench.json
exit $rc
