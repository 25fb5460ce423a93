"""Run-to-run stability of the captured PPO update (H1 x 8192 by default: 5 epochs x 4
mini-batches of the fused recurrent step; ROLL_TASK=go2 ROLL_ENVS=4096: the fused MLP step): after
two learning iterations, the update graph is
replayed N times from the same state (parameters, Adam moments and step, learning rate,
advantages restored before each replay), counting the replays whose parameters differ from the
first replay's.  None of the update's kernels uses atomics, so any difference is a race.
With the libppomlp.so named by PPOMLP_LIB.
usage: [PPOMLP_LIB=...] [ROLL_TASK=h1 ROLL_ENVS=8192] python tools/probes/update_race.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
TASK, NENV = os.environ.get("ROLL_TASK", "h1"), os.environ.get("ROLL_ENVS", "8192")
args = get_args(["--task", TASK, "--num_envs", NENV, "--headless"])
env, _ = task_registry.make_env(name=TASK, args=args)
r, _ = task_registry.make_alg_runner(env=env, name=TASK, args=args, log_root=None)
r.learn(2)  # the second iteration captures the update graph
alg = r.alg
st = alg.storage
if alg._rfused is not None:  # recurrent policies
    rf, graph = alg._rfused, alg._rgraph
    extra = []
else:  # the MLP step: also its bf16 weight copies (the Adam mirror rewrites them)
    rf, graph = alg._fused, alg._fgraph
    extra = [w for ws in rf.wb for w in ws] + ([w for ws in rf.wf for w in ws] if rf.wf else [])
assert rf is not None and graph is not None, "the fused update did not capture"
state = [rf.flat, rf.exp_avg, rf.exp_avg_sq, rf.step_t, alg._lr, st.advantages, st.returns] + extra
snap = [t.clone() for t in state]


def restore():
    for t, s in zip(state, snap):
        t.copy_(s)


restore()
graph.replay()
ref = rf.flat.clone()
bad = torch.zeros((), dtype=torch.int64, device=rf.flat.device)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(N):
    restore()
    graph.replay()
    bad += (rf.flat != ref).any().to(torch.int64)
    if i % 250 == 249:
        torch.cuda.synchronize()
        print(f"  {i + 1} updates, {int(bad)} differing", flush=True)
e1.record()
torch.cuda.synchronize()
print(f"{os.path.basename(os.environ.get('PPOMLP_LIB', 'libppomlp.so'))} {TASK}x{NENV}: {N} update replays, "
      f"{int(bad)} with parameters differing from the first ({e0.elapsed_time(e1) / N:.2f} ms per replay)",
      flush=True)
