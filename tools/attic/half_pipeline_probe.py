"""Probe: does splitting the rollout's envs into two halves on two streams hide the policy
forward behind the other half's env step?  (rollout.)

serial:     per step  fwd(4096 rows) -> k_step(4096 envs)            one stream
pipelined:  per step  fwd(2048) -> k_step(2048) on stream A, the same on stream B, no join
            between the streams inside the loop (eager and as one captured graph)
fwd is a torch MLP 48-512-256-128-12 (ELU) standing in for the fused rollout forward.
usage: python tools/probes/half_pipeline_probe.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402


def make(n):
    env, _ = task_registry.make_env(name="go2", args=get_args(["--task", "go2", "--num_envs", str(n), "--headless"]))
    env.reset()
    return env


def kstep(env):
    env.sim.step(env._env_structs[env._buf_idx], env.common_step_counter)


def main(T=48):
    full, ha, hb = make(4096), make(2048), make(2048)
    torch.manual_seed(0)
    mlp = torch.nn.Sequential(torch.nn.Linear(48, 512), torch.nn.ELU(), torch.nn.Linear(512, 256), torch.nn.ELU(),
                              torch.nn.Linear(256, 128), torch.nn.ELU(), torch.nn.Linear(128, 12)).cuda()
    xf, xa, xb = (torch.randn(n, 48, device="cuda") for n in (4096, 2048, 2048))
    q4 = [make(1024) for _ in range(4)]
    s4 = [torch.cuda.Stream() for _ in range(4)]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def serial():
        for _ in range(T):
            with torch.no_grad():
                full.actions.copy_(0.1 * torch.tanh(mlp(xf)))
            full.sim.set_stream(main_s.cuda_stream)
            kstep(full)

    def pipelined():
        sa.wait_stream(main_s)
        sb.wait_stream(main_s)
        for _ in range(T):
            for env, s, x in ((ha, sa, xa), (hb, sb, xb)):
                with torch.cuda.stream(s), torch.no_grad():
                    env.actions.copy_(0.1 * torch.tanh(mlp(x)))
                    env.sim.set_stream(s.cuda_stream)
                    kstep(env)
        main_s.wait_stream(sa)
        main_s.wait_stream(sb)

    M = [main_s]  # the stream the loops fork from and join into (the capture stream in a graph)

    def kstep_only(envs, streams):
        for s in streams:
            s.wait_stream(M[0])
        for _ in range(T):
            for env, s in zip(envs, streams):
                with torch.cuda.stream(s):
                    env.sim.set_stream(s.cuda_stream)
                    kstep(env)
        for s in streams:
            M[0].wait_stream(s)

    def kstep_joined(envs, streams):
        # every step: fork from main, one launch per stream, join back into main
        for _ in range(T):
            for env, s in zip(envs, streams):
                s.wait_stream(M[0])
                with torch.cuda.stream(s):
                    env.sim.set_stream(s.cuda_stream)
                    kstep(env)
            for s in streams:
                M[0].wait_stream(s)

    def graph_of(fn):
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        cap.wait_stream(main_s)
        torch.cuda.synchronize()
        M[0] = cap
        with torch.cuda.graph(g, stream=cap):
            fn()
        M[0] = main_s
        return g

    def fwd_only():
        for _ in range(T):
            with torch.no_grad():
                full.actions.copy_(0.1 * torch.tanh(mlp(xf)))

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(main_s)
            fn()
            b.record(main_s)
            torch.cuda.synchronize()
            best = min(best, a.elapsed_time(b) / T * 1e3)
        return best

    res = {
        "fwd_only(4096)": timeit(fwd_only),
        "kstep_only(4096)": timeit(lambda: kstep_only([full], [main_s])),
        "kstep_only(2048) one stream": timeit(lambda: kstep_only([ha], [sa])),
        "kstep_only(2x2048) two streams": timeit(lambda: kstep_only([ha, hb], [sa, sb])),
        "kstep_joined(2x2048) two streams": timeit(lambda: kstep_joined([ha, hb], [sa, sb])),
        "kstep_only(4x1024) four streams": timeit(lambda: kstep_only(q4, s4)),
        "kstep_joined(4x1024) four streams": timeit(lambda: kstep_joined(q4, s4)),
        "serial fwd+kstep(4096)": timeit(serial),
        "pipelined 2x(fwd+kstep(2048))": timeit(pipelined),
    }
    # the pipelined loop as one graph (fork/join on the two streams)
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(main_s)
    with torch.cuda.stream(cap):
        pipelined()  # warm on the capture stream
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cap):
        main_s_cap = torch.cuda.current_stream()
        sa.wait_stream(main_s_cap)
        sb.wait_stream(main_s_cap)
        for _ in range(T):
            for env, s, x in ((ha, sa, xa), (hb, sb, xb)):
                with torch.cuda.stream(s), torch.no_grad():
                    env.actions.copy_(0.1 * torch.tanh(mlp(x)))
                    env.sim.set_stream(s.cuda_stream)
                    kstep(env)
        main_s_cap.wait_stream(sa)
        main_s_cap.wait_stream(sb)
    gs = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gs, stream=cap):
        for _ in range(T):
            with torch.no_grad():
                full.actions.copy_(0.1 * torch.tanh(mlp(xf)))
            full.sim.set_stream(torch.cuda.current_stream().cuda_stream)
            kstep(full)
    res["graph serial fwd+kstep(4096)"] = timeit(gs.replay)
    for name, fn in (("graph kstep_only(4096)", lambda: kstep_only([full], [s4[0]])),
                     ("graph kstep_only(2x2048)", lambda: kstep_only([ha, hb], [sa, sb])),
                     ("graph kstep_joined(2x2048)", lambda: kstep_joined([ha, hb], [sa, sb])),
                     ("graph kstep_joined(4x1024)", lambda: kstep_joined(q4, s4))):
        res[name] = timeit(graph_of(fn).replay)
    res["graph pipelined 2x(fwd+kstep(2048))"] = timeit(g.replay)
    for k, v in res.items():
        print(f"{k:40s} {v:8.1f} us per step", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 48)
