# 128x128 GEMM tile-variant sweep of the fused optimizer step (per-launch timing, eager)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2 0 1 2; do
  PMLP_BIG_TILE=$v timeout -k 10 120 python tools/probes/update_step_time.py > gpurun_out/tile_$v.log 2>&1 || exit 1
  echo "variant $v" >> gpurun_out/tile_all.log; grep "us/step" gpurun_out/tile_$v.log >> gpurun_out/tile_all.log
done
echo done
