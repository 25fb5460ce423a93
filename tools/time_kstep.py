"""Time the fused env-step kernel (HIP events on its stream) for one or more builds.
usage: python tools/time_kstep.py [task] [num_envs] [lib.so ...]   (default: the shipped build)
TIME_KSTEP_ACTIONS=zero: zero actions (the robots stand on their feet: the same contact set for
every slot policy) instead of the default random flailing (0.5 N(0,1) actions, robots fall)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(task, n, lib):
    sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
    if lib:
        os.environ["LEGGEDSIM_LIB"] = lib
    import torch
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry  # noqa: F401
    from legged_gym.utils import get_args
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name=task, args=args)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    scale = 0.0 if os.environ.get("TIME_KSTEP_ACTIONS") == "zero" else 0.5
    acts = [scale * torch.randn(n, env.num_actions, device="cuda", generator=g) for _ in range(8)]
    for i in range(30):
        env.step(acts[i % 8])
    stream = torch.cuda.current_stream()
    K = 100
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
    print(f"{task} n={n} lib={os.path.basename(lib or 'default')} actions x{scale}: k_step median {ms[K // 2]:.4f} ms  "
          f"min {ms[0]:.4f}  -> {n / ms[K // 2] * 1e3:.3e} env-steps/s", flush=True)


if __name__ == "__main__":
    task = sys.argv[1] if len(sys.argv) > 1 else "go2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    libs = sys.argv[3:] or [""]
    if len(libs) == 1:
        run_one(task, n, libs[0])
    else:  # one process per build (the library is loaded once per process)
        for lib in libs:
            subprocess.run([sys.executable, __file__, task, str(n), lib], check=True)
