#!/bin/bash
# Per-phase cycle stamps of the fused env step for two stamp builds (e.g. this source and an
# earlier round's), same box.  usage: tools/gpu_stamps_ab.sh libA.so libB.so [task:n ...]
# log: gpurun_out/stamps_ab.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
A=$1; B=$2; shift 2
for p in ${@:-go2:4096 h1_2:8192}; do
  t=${p%%:*}; n=${p##*:}
  for lib in $A $B; do
    echo "== $lib" >> gpurun_out/stamps_ab.log
    LEGGEDSIM_LIB=$lib timeout -k 10 200 python tools/phase_stamps.py $t $n >> gpurun_out/stamps_ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/stamps_ab.log
