# The update's PPO loss inside the forward launch (pmlp_mlp_forward_ppo_loss, build/libppomlp_loss.so)
# against the shipped build: the full GPU suite on the new build, the captured-update time
# alternating (the new build with PMLP_FUSED_LOSS=0 too: the separate loss launch), and a bench run.
cd $GRAFT_REPO_ROOT
B=$PWD/unitree-rl-gym_amd/csrc/build
O=gpurun_out/ab_loss
mkdir -p $O
PPOMLP_LIB=$B/libppomlp_loss.so bash tools/gpu_tests.sh tests -m gpu -x || exit 1
cp gpurun_out/tests.log $O/tests.txt
for lib in libppomlp.so libppomlp_loss.so libppomlp.so libppomlp_loss.so libppomlp.so libppomlp_loss.so; do
  PPOMLP_LIB=$B/$lib timeout -k 10 200 python tools/probes/update_time.py $O/p_$lib.npz >> $O/update.txt 2>&1 || exit 2
done
PMLP_FUSED_LOSS=0 PPOMLP_LIB=$B/libppomlp_loss.so timeout -k 10 200 python tools/probes/update_time.py $O/p_sep.npz >> $O/update.txt 2>&1 || exit 3
PPOMLP_LIB=$B/libppomlp_loss.so timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 4
grep -E "update" $O/update.txt; tail -1 $O/tests.txt; python -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'])"
