"""Captured Go2 rollout (4096 envs, 24 steps: fused forward + k_step + k_step_extras per step)
with the libppomlp.so named by PPOMLP_LIB: median time of graph replays, and the rollout
storage + parameters after two seeded learning iterations digested (sha256) into argv[1] (for a bitwise
comparison of two builds, tools/gpu_rollout_ab.sh).
usage: [PPOMLP_LIB=...] [ROLL_DEFER=0] [ROLL_TASK=h1 ROLL_ENVS=8192] python tools/probes/rollout_time.py out.json"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402

TASK, NENV = os.environ.get("ROLL_TASK", "go2"), os.environ.get("ROLL_ENVS", "4096")
args = get_args(["--task", TASK, "--num_envs", NENV, "--headless"])
env, _ = task_registry.make_env(name=TASK, args=args)
_, train_cfg = task_registry.get_cfgs(TASK)
if os.environ.get("ROLL_DEFER") == "0":  # the env's own extras launch (runner cfg defer_env_extras)
    train_cfg.runner.defer_env_extras = False
r, _ = task_registry.make_alg_runner(env=env, name=TASK, args=args, train_cfg=train_cfg, log_root=None)
r.learn(2)  # the second iteration captures the rollout graph
assert r._rollout_graph is not None
torch.cuda.synchronize()
st = r.alg.storage
out = {k: getattr(st, k).detach().cpu().numpy() for k in ("actions", "actions_log_prob", "values", "mu", "rewards")}
out.update({f"p{i}": p.detach().cpu().numpy() for i, p in enumerate(r.alg.actor_critic.parameters())})
for name in ("saved_hidden_states_a", "saved_hidden_states_c"):  # (recurrent policies)
    for j, h in enumerate(getattr(st, name, None) or []):
        out[f"{name}{j}"] = h.detach().cpu().numpy()
if hasattr(st, "advantages"):
    out["advantages"], out["returns"] = st.advantages.detach().cpu().numpy(), st.returns.detach().cpu().numpy()
with open(sys.argv[1], "w") as f:  # a digest per array (the arrays themselves are ~100 MB per run)
    json.dump({k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() for k, v in out.items()}, f)
ts = []
with torch.inference_mode(False):
    for rnd in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            r._rollout_graph.graph.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 4)
ts.sort()
print(f"{os.path.basename(os.environ.get('PPOMLP_LIB', 'libppomlp.so'))} defer={os.environ.get('ROLL_DEFER', '1')} "
      f"tiles={os.environ.get('PMLP_LSTM_STEP_TILES', '-')} {TASK}x{NENV}: rollout {ts[len(ts) // 2]:.3f} ms median, "
      f"{ts[0]:.3f} min", flush=True)
