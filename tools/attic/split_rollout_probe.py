"""Probe: the Go2 rollout (24 captured steps: fused forward + k_step + k_step_extras) of 4096 envs
against two independent 2048-env rollouts replayed concurrently on two streams -- what an
env-halves pipelined rollout could gain at most (the halves never wait for each other).
usage: python tools/probes/split_rollout_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402


def runner(n):
    args = get_args(["--task", "go2", "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name="go2", args=args)
    r, _ = task_registry.make_alg_runner(env=env, name="go2", args=args, log_root=None)
    r.learn(2)  # the second iteration captures the rollout graph
    assert r._rollout_graph is not None
    return r


def main():
    full, ha, hb = runner(4096), runner(2048), runner(2048)
    main_s = torch.cuda.current_stream()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def one():
        full._rollout_graph.graph.replay()

    def one_half():
        ha._rollout_graph.graph.replay()

    def two():
        sa.wait_stream(main_s)
        sb.wait_stream(main_s)
        with torch.cuda.stream(sa):
            ha._rollout_graph.graph.replay()
        with torch.cuda.stream(sb):
            hb._rollout_graph.graph.replay()
        main_s.wait_stream(sa)
        main_s.wait_stream(sb)

    # both halves' 24 steps captured into ONE graph, each half on its own stream (fork at the
    # start, join at the end): what an env-halves rollout inside the runner's graph would be
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(main_s)
    torch.cuda.synchronize()
    state = {}
    for r in (ha, hb):
        state[id(r)] = (r._rollout_graph.obs, r._rollout_graph.critic_obs, r.env.common_step_counter,
                        r.alg.storage.step)
    with torch.inference_mode(False), torch.no_grad(), torch.cuda.graph(g, stream=cap):
        for r, s in ((ha, sa), (hb, sb)):
            s.wait_stream(cap)
            with torch.cuda.stream(s):
                obs, cobs, _, _ = state[id(r)]
                r.alg.storage.step = 0
                for t in range(r.num_steps_per_env):
                    obs, cobs, _, _, _ = r._collect_step(obs, cobs)
            cap.wait_stream(s)
    for r in (ha, hb):
        r.env.common_step_counter = state[id(r)][2]
        r.alg.storage.step = state[id(r)][3]

    def two_one_graph():
        g.replay()

    def timeit(fn, reps=10):
        with torch.inference_mode(False):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(main_s)
                fn()
                b.record(main_s)
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    for name, fn in (("rollout 4096 envs", one), ("rollout 2048 envs", one_half),
                     ("two 2048-env rollouts, two streams", two),
                     ("two 2048-env rollouts, one graph", two_one_graph), ("rollout 4096 envs (again)", one)):
        print(f"{name:40s} {timeit(fn):7.3f} ms per 24-step rollout", flush=True)


if __name__ == "__main__":
    main()
