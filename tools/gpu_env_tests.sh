# env GPU parity tests (incl. heightfield) + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_env.py -x -v --timeout 120 --timeout-method thread > gpurun_out/env_tests.log 2>&1 || exit 1
echo done
