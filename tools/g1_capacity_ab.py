"""G1 contact capacity A/B: G1 rough terrain at 4096 envs on the shipped
32-row kernel (8 contact slots, two envs per wave) against the 48-row kernel (12 contact slots,
one env per wave), same seeds and the same action sequence.  Reports per variant the capacity
drops per env-substep (lgs_get_contact_stats), the termination rate (resets that are not
time-outs) and the mean episode length at the end.
usage: python tools/g1_capacity_ab.py [steps] [task]   (one process per variant)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(variant, steps, task, scale):
    sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
    import torch
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry
    from legged_gym.utils import get_args
    cls = task_registry.get_task_class(task)
    if variant == "48":
        cls.max_contacts, cls.max_rows = 12, 48
    env, _ = task_registry.make_env(name=task, args=get_args(["--task", task, "--num_envs", "4096", "--headless"]))
    env.reset()
    env.sim.contact_stats(reset=True)
    g = torch.Generator(device="cuda").manual_seed(7)
    N = env.num_envs
    term = tout = 0
    a = torch.zeros(N, env.num_actions, device="cuda")
    for t in range(steps):
        a = 0.9 * a + scale * torch.randn(N, env.num_actions, device="cuda", generator=g)
        _, _, _, done, extras = env.step(a)
        to = env.time_out_buf
        term += int((done & ~to).sum())
        tout += int((done & to).sum())
    st = env.sim.contact_stats(reset=True)
    sub = steps * N * env.cfg.control.decimation
    print(f"{task} {variant}-row kernel ({env.max_contacts} slots): drops/env-substep bodies {st['bodies'] / sub:.2e} "
          f"self {st['self'] / sub:.2e} limits {st['limits'] / sub:.2e}; terminations {term / (steps * N):.4e} "
          f"per env-step, time-outs {tout}, mean episode length {float(env.episode_length_buf.float().mean()):.1f}",
          flush=True)


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    task = sys.argv[2] if len(sys.argv) > 2 else "g1_rough"
    if len(sys.argv) > 3:
        run(sys.argv[3], steps, task, float(sys.argv[4]))
    else:
        for scale in (0.1, 0.3):
            for variant in ("32", "48"):
                subprocess.run([sys.executable, __file__, str(steps), task, variant, str(scale)], check=True)
