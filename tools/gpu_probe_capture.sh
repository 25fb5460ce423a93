set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in randn act_value alg_act; do
  timeout -k 10 120 python tools/probes/rollout_capture.py $c >> gpurun_out/probe_capture.log 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/probe_capture.log
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
echo done
timeout -k 10 600 python -m pytest tests/test_gpu_env.py -x -q -m gpu -k "rollout_graph or training_smoke" > gpurun_out/pytest_rollout.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
