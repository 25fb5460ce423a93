import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch
import isaacgym  # noqa
from legged_gym.envs import task_registry
from legged_gym.utils import get_args
from legged_gym.utils.helpers import class_to_dict
from rsl_rl.runners import OnPolicyRunner
_, tc = task_registry.get_cfgs("go2")
args = get_args(["--task", "go2", "--num_envs", "256", "--headless"])
env, _ = task_registry.make_env(name="go2", args=args)
cfg = class_to_dict(tc); cfg["algorithm"]["schedule"] = "fixed"; cfg["algorithm"]["learning_rate"] = 3e-4
runner = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
runner.learn(2)
alg = runner.alg
def fin(name, ts): print(name, all(torch.isfinite(t).all().item() for t in ts), flush=True)
fin("params after learn(2)", list(alg.actor_critic.parameters()))
with torch.inference_mode():
    obs = env.get_observations()
    for _ in range(alg.storage.num_transitions_per_env):
        a = alg.act(obs, obs)
        obs, _, r, d, info = env.step(a)
        alg.process_env_step(r, d, info)
    alg.compute_returns(obs)
st = alg.storage
fin("storage", [st.observations, st.actions, st.rewards, st.values, st.returns, st.advantages, st.actions_log_prob, st.mu, st.sigma])
for variant in ("plain", "seed", "rngstate"):
    if variant == "seed": torch.manual_seed(5)
    if variant == "rngstate": torch.cuda.set_rng_state(torch.cuda.get_rng_state())
    st.step = st.num_transitions_per_env
    vl, sl = alg.update()
    print(variant, vl, sl, flush=True)
    fin(" params", list(alg.actor_critic.parameters()))
