# Fused-forward variants against the shipped build (NEW=build/<lib>, default libppomlp_epi.so:
# hidden outputs stored from the layer epilogue's registers): the fused-PPO GPU tests on the new
# build, the captured-update time alternating (tools/probes/update_time.py, parameters after 3
# updates compared bitwise) and the forward's phase clocks (tools/probes/fused_fwd_stamps.py,
# the matching -DPMLP_FMLP_STAMPS build <lib>_fstamps.so).
cd $GRAFT_REPO_ROOT
B=$PWD/unitree-rl-gym_amd/csrc/build
NEW=${NEW:-libppomlp_epi.so}
O=gpurun_out/ab_${NEW%.so}
mkdir -p $O
PPOMLP_LIB=$B/$NEW bash tools/gpu_tests.sh tests/test_gpu_fused_ppo.py -x || exit 1
cp gpurun_out/tests.log $O/tests.txt
for lib in libppomlp.so $NEW libppomlp.so $NEW libppomlp.so $NEW; do
  PPOMLP_LIB=$B/$lib timeout -k 10 200 python tools/probes/update_time.py $O/p_$lib.npz >> $O/update.txt 2>&1 || exit 2
done
NEW=$NEW python - >> $O/update.txt <<'PY'
import os
import numpy as np
o = "gpurun_out/ab_" + os.environ["NEW"][:-3]
a, b = np.load(f"{o}/p_libppomlp.so.npz"), np.load(f"{o}/p_{os.environ['NEW']}.npz")
print("params bitwise equal:", all(np.array_equal(a[k], b[k]) for k in a.files))
PY
PPOMLP_LIB=$B/${NEW%.so}_fstamps.so timeout -k 10 200 python tools/probes/fused_fwd_stamps.py > $O/stamps.txt 2>&1 || exit 3
grep -E "update|bitwise" $O/update.txt; grep -E "round 0|median" $O/stamps.txt
