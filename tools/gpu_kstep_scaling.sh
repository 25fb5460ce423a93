set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 256 1024 2048 4096 8192; do timeout -k 10 120 python tools/time_kstep.py go2 $n >> gpurun_out/kstep_scaling.log 2>&1 || exit 1; done
echo done
