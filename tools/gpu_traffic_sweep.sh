#!/bin/bash
# k_step HBM traffic vs env count: FETCH_SIZE and WRITE_SIZE passes
# (separate) of the shipped kernel and of the I/O-only diagnostic build (make iodiag: the
# step's global loads and stores without the physics, a known byte count per env) over an
# env-count sweep, then the linear fit bytes = intercept + slope * envs per build
# (tools/traffic_sweep_fit.py).  Needs build/libleggedsim_io.so pushed (.gpurunignore).
# usage: bash tools/gpu_traffic_sweep.sh [task] [envs ...]   (default: go2 512 1024 2048 4096)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TASK=${1:-go2}
shift
NS="${@:-512 1024 2048 4096}"
O=gpurun_out/traffic_sweep
[ "$TASK" = go2 ] || O=gpurun_out/traffic_sweep_$TASK
rm -rf $O && mkdir -p $O
B=unitree-rl-gym_amd/csrc/build
for lib in shipped io; do
  for n in $NS; do
    D=$O/${lib}_$n
    if [ $lib = io ]; then export LEGGEDSIM_LIB=$B/libleggedsim_io.so; else unset LEGGEDSIM_LIB; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python tools/profile_env.py $TASK $n 20 > $D.trace.log 2>&1 || exit 2
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python tools/profile_env.py $TASK $n 20 > $D.fetch.log 2>&1 || exit 3
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run --output-format csv -- python tools/profile_env.py $TASK $n 20 > $D.write.log 2>&1 || exit 4
    python tools/pmc_summary.py $D/trace $D/fetch $D/write "k_step<" $D/pmc_k_step.json > $D.pmc.log 2>&1 || exit 5
    find $D -name "*kernel_trace.csv" -delete; find $D -name "*counter_collection.csv" -size +2M -delete
    echo "$lib $n done"
  done
done
unset LEGGEDSIM_LIB
python tools/traffic_sweep_fit.py $O $O/fit.json $TASK > $O/fit.txt 2>&1 || exit 6
cat $O/fit.txt
