set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/probes/mlp4_time.py > gpurun_out/mlp4_time.log 2>&1 || exit 5
timeout -k 10 600 python -m pytest tests/test_gpu_fused_ppo.py -x -q > gpurun_out/pytest_fused.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python tools/ppo_timing.py > gpurun_out/ppo_timing.log 2>&1 || exit 3
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 4
echo done
