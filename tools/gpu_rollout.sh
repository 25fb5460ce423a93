# rollout-graph parity test + bench + per-phase timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_env.py -x -q -m gpu -k "rollout_graph or training_smoke" > gpurun_out/pytest_rollout.log 2>&1 || exit 1
timeout -k 10 300 python tools/ppo_timing.py > gpurun_out/ppo_timing.log 2>&1 || exit 3
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
echo done
