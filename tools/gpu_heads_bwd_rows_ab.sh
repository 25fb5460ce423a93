#!/bin/bash
# k_heads_bwd at 128 rows per workgroup (libppomlp.so) against 64 (libppomlp_b64.so, -DPMLP_HEADS_BWD_ROWS=64):
# the heads probe at the update's and the rollout's rows and the H1 x 8192 update replay, interleaved.
set -o pipefail
O=gpurun_out/b64; rm -rf $O; mkdir -p $O
B=$PWD/unitree-rl-gym_amd/csrc/build
for rep in 1 2; do for L in libppomlp.so libppomlp_b64.so; do
  PPOMLP_LIB=$B/$L timeout -k 10 120 python tools/probes/heads_time.py 49152 >> $O/ab.log 2>&1 || exit 1
  PPOMLP_LIB=$B/$L timeout -k 10 120 python tools/probes/heads_time.py 8192 >> $O/ab.log 2>&1 || exit 1
done; done
for L in libppomlp.so libppomlp_b64.so libppomlp.so libppomlp_b64.so; do
  PPOMLP_LIB=$B/$L timeout -k 10 300 python tools/probes/update_race.py 300 > $O/upd.log 2>&1 || exit 1
  grep "update replays" $O/upd.log >> $O/ab.log
done
grep -v amdgpu.ids $O/ab.log
