"""A/B: the humanoid env step at its 48-row capacity (12 contacts, one env per wave)
against the 32-row capacity (8 contacts: two envs per wave where the build has that
variant).  Times k_step with HIP events on the env's stream and reports the active
contact statistics the kernel's outputs imply (feet with force, per step).
usage: python tools/probes/humanoid_rows_ab.py task:num_envs:max_contacts:max_rows ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_one(task, n, mc, mr):
    sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
    import torch
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry  # noqa: F401
    from legged_gym.envs.base.humanoid import HumanoidRobot
    from legged_gym.utils import get_args
    HumanoidRobot.max_contacts, HumanoidRobot.max_rows = mc, mr
    HumanoidRobot.max_self_contacts = min(HumanoidRobot.max_self_contacts, mc)
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name=task, args=args)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [0.3 * torch.randn(n, env.num_actions, device="cuda", generator=g) for _ in range(8)]
    for i in range(60):
        env.step(acts[i % 8])
    stream = torch.cuda.current_stream()
    K = 60
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    torch.cuda.synchronize()
    for i in range(K):
        env._buf_idx ^= 1
        env.actions.copy_(acts[i % 8])
        ev[i][0].record(stream)
        env.sim.step(env._env_structs[env._buf_idx], env.common_step_counter)
        ev[i][1].record(stream)
        env.account_replayed_steps(1)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    cf = env.contact_forces[:, env.feet_indices, 2]
    feet_down = (cf > 1.0).float().sum(1).mean().item()
    print(f"{task} n={n} contacts={mc} rows={mr} epw={getattr(env.sim, 'epw', '?')}: k_step median "
          f"{ms[K // 2]:.4f} ms min {ms[0]:.4f}; feet with force {feet_down:.2f}; "
          f"resets/step {env.reset_buf.float().mean().item():.4f}", flush=True)


if __name__ == "__main__":
    for spec in sys.argv[1:]:
        if len(sys.argv) > 2:
            subprocess.run([sys.executable, __file__, spec], check=True)
        else:
            t, n, mc, mr = spec.split(":")
            run_one(t, int(n), int(mc), int(mr))
