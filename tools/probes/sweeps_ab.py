"""k_step time against the contact solve's sweep count (cfg.sim.physx.pgs_sweeps), one process
per setting, alternating, median of 100 launches each (as tools/time_kstep.py).
usage: python tools/probes/sweeps_ab.py task num_envs rounds sweeps [sweeps ...]"""
import copy
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_one(task, n, sweeps):
    sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
    import torch
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry
    from legged_gym.utils import get_args
    env_cfg, _ = task_registry.get_cfgs(task)
    env_cfg = copy.deepcopy(env_cfg)
    env_cfg.sim.physx.pgs_sweeps = sweeps
    env, _ = task_registry.make_env(name=task, args=get_args(["--task", task, "--num_envs", str(n), "--headless"]),
                                    env_cfg=env_cfg)
    assert env._lgs_params.solver_iterations == sweeps
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g) for _ in range(8)]
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
    print(f"{task} n={n} sweeps={sweeps}: k_step median {ms[K // 2]:.4f} ms  min {ms[0]:.4f}", flush=True)


if __name__ == "__main__":
    task, n = sys.argv[1], int(sys.argv[2])
    if len(sys.argv) == 4:
        run_one(task, n, int(sys.argv[3]))
    else:
        rounds, sweeps = int(sys.argv[3]), [int(x) for x in sys.argv[4:]]
        for _ in range(rounds):
            for sw in sweeps:
                subprocess.run([sys.executable, __file__, task, str(n), str(sw)], check=True)
