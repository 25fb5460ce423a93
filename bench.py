"""Benchmark: env-steps/s + PPO-iteration wall time, Go2, 4096 envs per GPU.

A bench "step" is one rsl_rl PPO iteration (BASELINE.json metric): 24 control
steps of the 4096-env Go2 task (policy inference + the fused HIP env step) and
the PPO update (5 epochs x 4 mini-batches), exactly what OnPolicyRunner.learn
does per iteration.  value = env-steps/s over the whole job
(= n_gpus * 4096 * 24 * K / max-over-ranks wall time); ms_per_step = the
PPO-iteration wall time.

Multi-GPU: launched by torch.distributed.run, one process per GPU; envs are
sharded (4096 per rank, weak scaling) and PPO all-reduces one flat gradient
bucket per optimizer step over RCCL.

Extra fields: env-only and rollout throughput, the live-timed fused env-step
kernel against the HBM roofline (algorithmic bytes), and the CPU
oracle baseline (rank 0, N=1 only).
"""
import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))

NUM_ENVS = 4096
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# algorithmic bytes per Go2 env-step (state read+write, obs, rewards, ...)
GO2_BYTES_PER_ENV_STEP = 1154


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10, help="timed PPO iterations")
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--num_envs", type=int, default=NUM_ENVS)
    p.add_argument("--env_steps", type=int, default=200, help="timed control steps of the env-only leg")
    p.add_argument("--cpu_seconds", type=float, default=12.0, help="budget of the CPU oracle baseline")
    p.add_argument("--no_cpu_baseline", action="store_true")
    p.add_argument("--no_other_configs", action="store_true",
                   help="skip the env-only legs of BASELINE configs[2..4] (G1 heightfield, H1, H1_2)")
    return p.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args):
    """`bench.py --gpus N` (N > 1) outside a launcher: start N ranks of this script under
    torch.distributed.run, one process per GPU, and exit with their status.  Runs before
    anything touches the GPU (no HIP call in this parent process)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


@contextlib.contextmanager
def _stdout_fd_to_stderr():
    """File descriptor 1 onto 2 for the block: Python prints and native libraries' writes alike."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def setup_dist(args):
    """This rank's world, rank and device through the package's own launcher hook
    (legged_gym.utils.distributed.init_from_env, the one train.py uses): RCCL when every rank
    owns a GPU, gloo when ranks share one; LEGGED_GYM_DIST_BACKEND overrides."""
    import torch
    from legged_gym.utils.distributed import init_from_env, rank_device, world_from_env
    world, rank, local, _ = world_from_env()
    with _stdout_fd_to_stderr():  # stdout carries only the JSON line (gloo's C++ connect log too)
        world = init_from_env(None)
    dev = f"cuda:{rank_device(local, torch.cuda.device_count())}"
    torch.cuda.set_device(dev)
    return world, rank, dev


def barrier(world):
    import torch.distributed as dist
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    # gloo reduces host tensors; RCCL device tensors
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([x], device="cuda" if on_dev else "cpu", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# the committed rocprofv3 summaries of the current build (tools/gpu_env_profile.sh; the
# newest round that has them)
PROFILE_DIR = next((d for d in (os.path.join(ROOT, "profiles", r, "env_go2_4096") for r in ("round6", "round5", "round4", "round3"))
                    if os.path.exists(os.path.join(d, "pmc_k_step.json"))),
                   os.path.join(ROOT, "profiles", "round3", "env_go2_4096"))


def load_pmc():
    """HBM bytes per launch of the env-step kernel from the committed rocprofv3 PMC summary
    (FETCH_SIZE / WRITE_SIZE in separate passes: tools/pmc_summary.py), or None.  Where the
    known-byte calibration of the I/O-only diagnostic build is committed
    (traffic_calib.json, tools/traffic_calib.py: the counters' tally factor for this kernel's
    own access pattern), its bytes are the traffic; else the 1 GiB-copy calibration's."""
    try:
        with open(os.path.join(PROFILE_DIR, "pmc_k_step.json")) as f:
            d = json.load(f)
    except Exception:
        return None
    try:
        with open(os.path.join(PROFILE_DIR, "traffic_calib.json")) as f:
            k = json.load(f)["k_step"]
        d["copy_calibrated_bytes_per_launch"] = d.get("hbm_bytes_per_launch")
        d["hbm_bytes_per_launch"] = k["hbm_bytes_per_launch"]
        d["read_bytes_per_launch"], d["write_bytes_per_launch"] = k["read_bytes_per_launch"], k["write_bytes_per_launch"]
        d["calibration"] = "known-byte I/O-only build (traffic_calib.json)"
    except Exception:
        d["calibration"] = "1 GiB copy in the same pass"
    return d


# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per
# SIMD (MI355X_MICROARCH.md: 32 lanes/cycle), at the 2.4 GHz peak engine clock
VALU_PEAK_GINST_S = 256 * 4 * 2.4 / 2


def load_sq_valu(kernel_ms):
    """VALU-issue roofline of the env-step kernel: instructions per launch from the committed
    rocprofv3 SQ summary (profiles/sq_k_step.json, tools/sq_summary.py) over the live launch
    time.  The env step is latency-bound, so this, not GB/s, is its meaningful
    utilisation figure; reported beside the HBM roofline the contract asks for."""
    path = os.path.join(PROFILE_DIR, "sq_k_step.json")
    try:
        with open(path) as f:
            sq = json.load(f)
    except Exception:
        return None
    ginst = sq["valu_insts_per_launch"] / (kernel_ms * 1e-3) / 1e9
    return {"achieved": round(ginst, 1), "peak": VALU_PEAK_GINST_S, "unit": "G VALU inst/s", "frac": ginst / VALU_PEAK_GINST_S,
            "valu_insts_per_launch": sq["valu_insts_per_launch"], "share_of_wave_time": sq.get("share_of_wave_time")}


def load_wave_timeline():
    """The env-step launch's wave timeline from the committed stamps-build summary
    (profiles/round5/env_go2_4096/wave_timeline.txt, tools/wave_timeline.py): the launch ends
    with its slowest wave, so the median wave's duration against the span is the share of the
    launch the per-step barrier costs."""
    import re
    try:
        txt = open(os.path.join(PROFILE_DIR, "wave_timeline.txt")).read()
        span = float(re.search(r"launch span ([\d.]+) us", txt).group(1))
        med = float(re.search(r"median ([\d.]+) p90", txt).group(1))
        mx = float(re.search(r"p90 [\d.]+ max ([\d.]+)", txt).group(1))
    except Exception:
        return None
    return {"median_wave_us": med, "max_wave_us": mx, "span_us": span, "median_over_span": round(med / span, 3),
            "source": os.path.relpath(os.path.join(PROFILE_DIR, "wave_timeline.txt"), ROOT)}


def _cpu_share():
    """The CPUs this process may use: its affinity mask and the cgroup v2 cpu.max quota."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    return {"affinity_cpus": aff, "cgroup_quota_cpus": quota}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_rate(env, bridge, lib, n_envs, seconds, threads):
    """env-steps/s of the oracle's fused step (PD + substeps + post-physics) over n_envs
    copies of the env's state, with `threads` OpenMP threads."""
    import ctypes
    import numpy as np
    gomp = ctypes.CDLL("libgomp.so.1")
    gomp.omp_set_num_threads(int(threads))
    snap = bridge.snapshot(env)
    reps = -(-n_envs // env.num_envs)
    b = {}
    for k, v in snap.items():
        if v is None:
            b[k] = None
        elif k in ("episode_sums",):
            b[k] = np.ascontiguousarray(np.tile(v, (1, reps))[:, :n_envs])
        elif k in ("episode_acc",):
            b[k] = v.copy()
        else:
            rows = v.reshape(env.num_envs, -1)
            b[k] = np.ascontiguousarray(np.tile(rows, (reps, 1))[:n_envs].reshape((-1,) + v.shape[1:]))
    rng = np.random.default_rng(0)
    acts = [rng.normal(0, 0.5, (n_envs, env.num_actions)).astype(np.float32) for _ in range(4)]
    steps, t0 = 0, time.time()
    while True:
        b["actions"][:] = acts[steps % 4]
        b["episode_acc"][:] = 0
        bridge.step_raw(env.model, env._lgs_params, env.task_params, n_envs, b, 10_000 + steps, lib)
        steps += 1
        el = time.time() - t0
        if el >= seconds and steps >= 2:
            break
    return n_envs * steps / el, steps, el


def _cpu_ppo_iter_s(num_envs, obs_dim, num_actions, threads, env_step_rate, sample_steps=2):
    """PPO iteration on the host: 24 x (policy inference on CPU torch + the oracle env step
    at env_step_rate) + the update (5 epochs x 4 mini-batches; `sample_steps` optimizer steps
    timed and scaled to the 20).  Go2 MLP actor-critic 512-256-128, fp32 CPU torch."""
    import torch
    from rsl_rl.algorithms import PPO
    from rsl_rl.modules import ActorCritic
    torch.set_num_threads(int(threads))
    T, epochs, mbs = 24, 5, 4
    with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON line
        ac = ActorCritic(obs_dim, obs_dim, num_actions, [512, 256, 128], [512, 256, 128], mixed_precision=False)
    ppo = PPO(ac, num_learning_epochs=epochs, num_mini_batches=mbs, learning_rate=1e-3, schedule="adaptive",
              desired_kl=0.01, entropy_coef=0.01, device="cpu", fused_loss=False)
    opt = ppo.optimizer
    obs = torch.randn(num_envs, obs_dim)
    with torch.no_grad():
        ac.act_and_value(obs, obs)
        t0 = time.time()
        for _ in range(T):
            ac.act_and_value(obs, obs)
        infer = time.time() - t0
    rows = num_envs * T // mbs
    g = torch.Generator().manual_seed(0)
    xb = torch.randn(rows, obs_dim, generator=g)
    mu = 0.3 * torch.randn(rows, num_actions, generator=g)
    sigma = torch.ones(rows, num_actions)
    ab = mu + torch.randn(rows, num_actions, generator=g)
    logp = torch.distributions.Normal(mu, sigma).log_prob(ab).sum(-1, keepdim=True)
    val, adv, ret = (torch.randn(rows, 1, generator=g) for _ in range(3))
    t0 = time.time()
    for _ in range(sample_steps):  # rsl_rl v1.0.2's PPO loss (the torch statement, PPO._reference_loss)
        loss, _, _ = ppo._reference_loss(xb, xb, ab, val, adv, ret, logp, mu, sigma, (None, None), None)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(ac.parameters(), 1.0)
        opt.step()
    upd = (time.time() - t0) / sample_steps * epochs * mbs
    return T * num_envs / env_step_rate + infer + upd, infer, upd


def cpu_baseline(env, seconds):
    """The CPU oracle (oracle/lgs_oracle.c, OpenMP over envs) on the same Go2 workload, plus
    the policy and the PPO update on CPU torch: Go2 4096 and 4 envs,
    all host threads of this job and 1 thread."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import subprocess
    import bridge
    from leggedsim import cabi
    # the oracle compiled for this host's CPU (-march=native); the portable x86-64-v3 build
    # that travels with the tree if the host compiler is unavailable
    build = "gcc -O3 -march=native -ffp-contract=off -fopenmp, built on this host (oracle/Makefile native)"
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True, timeout=180,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        lib = cabi.load_oracle(os.path.join(ROOT, "oracle", "_build", "liblgs_oracle_native.so"))
    except Exception:
        lib = bridge.ensure_built()
        build = ("gcc -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp (oracle/Makefile; built in the container, "
                 "the native build failed on this host)")
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    share = _cpu_share()
    n = env.num_envs
    half = max(2.0, seconds / 4)
    rate_all, st_all, el_all = _oracle_rate(env, bridge, lib, n, half, threads)
    rate_one, st_one, el_one = _oracle_rate(env, bridge, lib, n, half, 1)
    rate4_all, _, _ = _oracle_rate(env, bridge, lib, 4, 1.0, threads)
    rate4_one, _, _ = _oracle_rate(env, bridge, lib, 4, 1.0, 1)
    it_all, inf_all, upd_all = _cpu_ppo_iter_s(n, env.num_obs, env.num_actions, threads, rate_all)
    it4, _, _ = _cpu_ppo_iter_s(4, env.num_obs, env.num_actions, threads, rate4_all, sample_steps=5)
    import torch
    torch.set_num_threads(threads)
    return {"value": round(24 * n / it_all, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": (f"Go2 {n} envs: oracle fused step (PD + 4 substeps + post-physics) {st_all} steps in "
                       f"{el_all:.1f} s on {threads} threads; PPO iteration = 24 x (oracle step + CPU torch "
                       f"MLP policy) + update (2 optimizer steps of rsl_rl's PPO loss on 24,576 rows, clip_grad_norm_ and "
                       f"Adam timed, scaled to 5 x 4)"),
            "ppo_iter_ms": round(it_all * 1e3, 1),
            "ppo_iter_breakdown_ms": {"env": round(24 * n / rate_all * 1e3, 1), "inference": round(inf_all * 1e3, 1),
                                      "update": round(upd_all * 1e3, 1)},
            "env_only_env_steps_per_s": round(rate_all, 1),
            "env_only_env_steps_per_s_1_thread": round(rate_one, 1),
            "go2_4_envs": {"env_only_env_steps_per_s": round(rate4_all, 1),
                           "env_only_env_steps_per_s_1_thread": round(rate4_one, 1),
                           "ppo_iter_ms": round(it4 * 1e3, 2)},
            "host_cpu": _cpu_model(), "nproc": os.cpu_count(), "cpu_share": share,
            "cores_note": (f"{threads} threads = OMP_NUM_THREADS, the job's CPU share as the harness sets it; "
                           f"the process may run on {share['affinity_cpus']} CPUs (sched_getaffinity), cgroup "
                           f"cpu.max quota {share['cgroup_quota_cpus']} CPUs; nproc counts the whole machine"),
            "build": build}


def ppo_iter_rate(task, n, dev, iters, warmup, get_args, task_registry):
    """PPO iterations (OnPolicyRunner.learn: captured rollout + GAE + captured update) of
    another BASELINE config with its own policy (G1 / H1 / H1_2: ActorCriticRecurrent,
    LSTM 64, on the HIP sequence kernels): ms per iteration and env-steps/s."""
    import torch
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    gargs = get_args(["--task", task, "--num_envs", str(n), "--headless", "--sim_device", dev, "--rl_device", dev])
    with contextlib.redirect_stdout(sys.stderr):
        env, env_cfg = task_registry.make_env(name=task, args=gargs)
        _, train_cfg = task_registry.get_cfgs(task)
        runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device=dev)
        runner.learn(num_learning_iterations=warmup, init_at_random_ep_len=True)
    torch.cuda.synchronize(dev)
    t0 = time.time()
    with contextlib.redirect_stdout(sys.stderr):
        runner.learn(num_learning_iterations=iters)
    torch.cuda.synchronize(dev)
    el = time.time() - t0
    T = runner.num_steps_per_env
    out = {"num_envs": n, "policy": runner.cfg["policy_class_name"], "decimation": env_cfg.control.decimation,
           "ppo_iter_ms": round(el / iters * 1e3, 3), "env_steps_per_s": round(n * T * iters / el, 1),
           "rollout_graph": runner._rollout_graph is not None,
           "update_graph": any(getattr(runner.alg, g, None) is not None for g in ("_graph", "_fgraph", "_rgraph")),
           "update_path": "fused recurrent step" if getattr(runner.alg, "_rfused", None) is not None else
           ("fused MLP step" if getattr(runner.alg, "_fused", None) is not None else "autograd"),
           "domain_rand": bool(env_cfg.domain_rand.randomize_friction or env_cfg.domain_rand.randomize_base_mass),
           "terrain": env_cfg.terrain.mesh_type, "iters_timed": iters}
    env.close()
    return out


def capacity_drops(env, steps):
    """What the fixed constraint capacity (8 contact slots + 8 limit rows per env) left out over
    the last `steps` control steps (lgs_get_contact_stats), per env and substep: touching bodies
    without a contact row, self contacts without one, violated joint limits without a row."""
    st = env.sim.contact_stats(reset=True)
    den = float(steps * env.num_envs * env.cfg.control.decimation)
    return {k: v / den for k, v in st.items()}


def env_kernel_rate(task, n, dev, steps, get_args, task_registry):
    """Back-to-back fused env steps of another BASELINE config (env only, no policy),
    timed with HIP events on the env's stream: env-steps/s and ms per step."""
    import torch
    gargs = get_args(["--task", task, "--num_envs", str(n), "--headless", "--sim_device", dev, "--rl_device", dev])
    with contextlib.redirect_stdout(sys.stderr):
        env, _ = task_registry.make_env(name=task, args=gargs)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(0)
    acts = [0.5 * torch.randn(n, env.num_actions, device=dev, generator=g) for _ in range(4)]
    for i in range(10):
        env.step(acts[i % 4])
    stream = torch.cuda.current_stream(dev)
    env._sync_stream()
    env.actions.copy_(acts[0])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    env.sim.contact_stats(reset=True)
    e0.record(stream)
    for i in range(steps):
        env._buf_idx ^= 1
        env.sim.step(env._env_structs[env._buf_idx], env.common_step_counter)
        env.account_replayed_steps(1)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    out = {"num_envs": n, "decimation": env.cfg.control.decimation, "env_step_kernel_ms": round(ms, 4),
           "env_steps_per_s": round(n / (ms * 1e-3), 1),
           "terrain": env.cfg.terrain.mesh_type,
           "capacity_drops_per_env_substep": capacity_drops(env, steps)}
    env.close()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    import torch
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry  # noqa: F401  (before legged_gym.utils: the registry's import order)
    world, rank, dev = setup_dist(args)
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    from legged_gym.utils import get_args
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner

    gargs = get_args(["--task", "go2", "--num_envs", str(args.num_envs), "--headless", "--sim_device", dev,
                      "--rl_device", dev])
    with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON line
        env, env_cfg = task_registry.make_env(name="go2", args=gargs)
        _, train_cfg = task_registry.get_cfgs("go2")
        runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device=dev)
    T = runner.num_steps_per_env
    N = env.num_envs

    # ---- env-only leg: the fused step kernel, timed with HIP events on its stream
    g = torch.Generator(device=dev).manual_seed(rank)
    acts = [0.5 * torch.randn(N, env.num_actions, device=dev, generator=g) for _ in range(8)]
    for i in range(20):
        env.step(acts[i % 8])
    stream = torch.cuda.current_stream(dev)
    env._sync_stream()
    # (a) back-to-back lgs_step launches (k_step + its one-block extras kernel) between two
    #     HIP events on the env's stream: the per-launch device time of the fused step
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    env.actions.copy_(acts[0])
    torch.cuda.synchronize(dev)
    env.sim.contact_stats(reset=True)
    e0.record(stream)
    for i in range(args.env_steps):
        env._buf_idx ^= 1
        env.sim.step(env._env_structs[env._buf_idx], env.common_step_counter)
        env.account_replayed_steps(1)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = e0.elapsed_time(e1) / args.env_steps
    go2_drops = capacity_drops(env, args.env_steps)
    # (b) env.step() as the runner calls it (actions copy + launch + extras dict)
    t0 = time.time()
    for i in range(args.env_steps):
        env.step(acts[i % 8])
    torch.cuda.synchronize(dev)
    env_wall = time.time() - t0
    env_only = N * args.env_steps / env_wall

    # ---- rollout leg: policy inference + env.step (no update)
    with torch.inference_mode():
        obs = env.get_observations()
        for _ in range(10):
            obs, _, _, _, _ = env.step(runner.alg.actor_critic.act(obs))
        torch.cuda.synchronize(dev)
        t0 = time.time()
        for _ in range(2 * T):
            obs, _, _, _, _ = env.step(runner.alg.actor_critic.act(obs))
        torch.cuda.synchronize(dev)
    rollout = N * 2 * T / (time.time() - t0)

    # ---- full PPO iterations (the metric)
    runner.learn(num_learning_iterations=args.warmup, init_at_random_ep_len=True)
    torch.cuda.synchronize(dev)
    barrier(world)
    t0 = time.time()
    runner.learn(num_learning_iterations=args.steps)
    torch.cuda.synchronize(dev)
    barrier(world)
    elapsed = max_over_ranks(time.time() - t0, world)
    ms_per_iter = elapsed / args.steps * 1e3
    value = world * N * T * args.steps / elapsed

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    bytes_per_launch = GO2_BYTES_PER_ENV_STEP * N
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    pmc = load_pmc() or {}
    line = {
        "metric": "env-steps/sec + PPO-iter wall-time, Go2 4096 envs/GPU at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_iter, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32 env step; bf16 MFMA policy GEMMs (fp32 accumulate)",
        "data": "synthetic (random-init policy, simulated Go2 on flat ground)",
        "config": {"workload": "Go2 flat terrain, 4096 envs/GPU, MLP actor-critic 512-256-128, PPO 24 steps x 5 epochs x 4 mini-batches",
                   "num_envs_per_gpu": N, "decimation": env_cfg.control.decimation,
                   "parallelism": f"dp{world}"},
        "ppo_iter_ms": round(ms_per_iter, 3),
        "env_only_env_steps_per_s": round(env_only, 1),
        "rollout_env_steps_per_s": round(rollout, 1),
        "env_step_kernel_ms": round(kernel_ms, 4),
        "capacity_drops_per_env_substep": go2_drops,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": pmc.get("hbm_bytes_per_launch"),
                     "traffic_read_write": [pmc.get("read_bytes_per_launch"), pmc.get("write_bytes_per_launch")],
                     "traffic_profile_avg_ns": pmc.get("avg_ns"), "traffic_calibration": pmc.get("calibration"),
                     "traffic_profile": os.path.relpath(PROFILE_DIR, ROOT),
                     "kernel": pmc.get("kernel", "k_step (fused Go2 control step)"),
                     "algorithmic_bytes_per_launch": bytes_per_launch, "valu": load_sq_valu(kernel_ms),
                     "waves": load_wave_timeline()},
    }
    if world == 1 and not args.no_other_configs:
        # the other BASELINE configs on this GPU (not this line's metric): G1 rough heightfield
        # 4096, H1 8192, H1_2 8192 (+DR, decimation 8) -- the fused env step alone, and the
        # whole PPO iteration with their recurrent (LSTM) policies
        line["other_configs_env_only"] = {
            "g1_rough_heightfield_4096": env_kernel_rate("g1_rough", 4096, dev, 50, get_args, task_registry),
            "h1_8192": env_kernel_rate("h1", 8192, dev, 50, get_args, task_registry),
            "h1_2_8192": env_kernel_rate("h1_2", 8192, dev, 50, get_args, task_registry),
        }
        line["other_configs_ppo_iter"] = {
            # configs[0]: the reference's CPU-runnable case (Go2, 4 envs) on this GPU
            "go2_4": ppo_iter_rate("go2", 4, dev, 5, 2, get_args, task_registry),
            "g1_rough_heightfield_4096": ppo_iter_rate("g1_rough", 4096, dev, 3, 2, get_args, task_registry),
            "h1_8192": ppo_iter_rate("h1", 8192, dev, 3, 2, get_args, task_registry),
            "h1_2_8192": ppo_iter_rate("h1_2", 8192, dev, 3, 2, get_args, task_registry),
        }
        line["h1_2_8192_ppo_iter_ms"] = line["other_configs_ppo_iter"]["h1_2_8192"]["ppo_iter_ms"]
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(env, args.cpu_seconds)
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
