# PARTIAL_TN (row-major activations only) vs transposed copies: kernel + update tests,
# interleaved update A/B, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_ppo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tn_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/probes/update_env_ab.py PMLP_TN 1 0 > gpurun_out/tn_ab.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --no_other_configs > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3
tail -2 gpurun_out/tn_ab.log
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['env_step_kernel_ms'])"
echo done
