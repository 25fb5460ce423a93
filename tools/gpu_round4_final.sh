# Round-4 closing measurements of the shipped build, one box: the full GPU suite, smoke, the
# default bench line and the profile sets of the given configs (tools/gpu_round4_profile.sh).
# Every step under its own time limit; the first failure ends the script.
# usage: bash tools/gpu_round4_final.sh [task:envs ...]   (default go2:4096)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final2
mkdir -p $O
bash tools/gpu_tests.sh tests -m gpu; rc=$?; cp gpurun_out/tests.log $O/gpu_tests.txt; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 3
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 4
bash tools/gpu_round4_profile.sh ${@:-go2:4096} || exit 5
echo final2 done
