"""Per-control-step time of the fused env step launched once per step (the shipped build)
against 24 steps per launch (make -C unitree-rl-gym_amd/csrc multidiag: the same step looped
inside k_step, no kernel boundary between the steps) -- the cost of the per-launch barrier
(a launch ends with its slowest wave).  Random actions held for the whole
measurement.  usage: python tools/probes/multistep_probe.py [task] [num_envs]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MULTI = os.path.join(ROOT, "unitree-rl-gym_amd", "csrc", "build", "libleggedsim_multi.so")


def run(task, n, lib):
    sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
    if lib:
        os.environ["LEGGEDSIM_LIB"] = lib
    import torch
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry  # noqa: F401
    from legged_gym.utils import get_args
    env, _ = task_registry.make_env(name=task, args=get_args(["--task", task, "--num_envs", str(n), "--headless"]))
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    env.actions.copy_(0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g))
    per = 24 if lib else 1
    K = 96 // per
    stream = torch.cuda.current_stream()
    for _ in range(3):
        env.sim.step(env._env_structs[env._buf_idx], env.common_step_counter)
    torch.cuda.synchronize()
    res = []
    for rep in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(K):
            env.sim.step(env._env_structs[env._buf_idx], env.common_step_counter)
        b.record(stream)
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / (K * per))
    res.sort()
    print(f"{task} n={n} {'24 steps per launch' if lib else 'one step per launch'}: {res[2]:.1f} us per control "
          f"step (median of 5 x {K * per} steps; min {res[0]:.1f})", flush=True)


if __name__ == "__main__":
    task = sys.argv[1] if len(sys.argv) > 1 else "go2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    if len(sys.argv) > 3:
        run(task, n, sys.argv[3] if sys.argv[3] != "default" else "")
    else:
        for rep in range(2):
            for lib in ("default", MULTI):
                subprocess.run([sys.executable, __file__, task, str(n), lib], check=True)
