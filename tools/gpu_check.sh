#!/bin/bash
# One box, the shipped build: the GPU suite (args: pytest selection, default the whole -m gpu
# suite), smoke, and the default bench line, into gpurun_out/$OUT (default check).  Every
# step under its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${OUT:-check}
mkdir -p $O
bash tools/gpu_tests.sh ${@:-tests} -m gpu; rc=$?; cp gpurun_out/tests.log $O/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 3
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 4
cat $O/bench.json
