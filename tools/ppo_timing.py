"""Time collection vs update of OnPolicyRunner on Go2 x 4096, plus the env-only and
policy-only parts of a rollout step (where the collection time goes)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402

args = get_args(["--task", "go2", "--num_envs", "4096", "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
_, tc = task_registry.get_cfgs("go2")
runner = OnPolicyRunner(env, class_to_dict(tc), log_dir=None, device="cuda:0")
runner.sync_phase_times = True  # device-exact phase times
runner.learn(3)
cs, ls = [], []
for _ in range(5):
    runner.learn(1)
    c, l = runner.last_iteration_times
    cs.append(c)
    ls.append(l)
print(f"collection {1e3 * sum(cs) / 5:.2f} ms, learn {1e3 * sum(ls) / 5:.2f} ms", flush=True)
obs = env.get_observations()
alg = runner.alg
with torch.inference_mode():
    for name, fn in (("env.step", lambda o: env.step(alg.actor_critic.act_inference(o))[0]),
                     ("alg.act", lambda o: (alg.act(o, o), o)[1]),
                     ("act+step+store", lambda o: (lambda a: (lambda r: (alg.process_env_step(r[2], r[3], r[4]), r[0])[1])(env.step(a)))(alg.act(o, o)))):
        for _ in range(3):
            obs = fn(obs)
        alg.storage.clear()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(24):
            obs = fn(obs)
        cpu = time.time() - t0
        torch.cuda.synchronize()
        alg.storage.clear()
        print(f"{name:16s}: {1e3 * (time.time() - t0) / 24:.3f} ms/step (host issue {1e3 * cpu / 24:.3f})", flush=True)
