# split-K slab count sweep of the fused optimizer step's weight-gradient GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "256 1024" "512 256" "1024 256" "512 128" "1024 128"; do
  set -- $cfg
  PMLP_SPLIT_TARGET=$1 PMLP_SPLIT_MIN_ROWS=$2 timeout -k 10 120 python tools/probes/update_step_time.py > gpurun_out/split_$1_$2.log 2>&1 || exit 1
done
echo done
