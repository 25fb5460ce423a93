"""Data-parallel recurrent PPO update (BASELINE configs[3]/[4]: H1 / H1_2 train
ActorCriticRecurrent with one process per GPU): shared by the CPU (gloo) and GPU tests.

A synthetic rollout of 2N envs is built on the host (identical in every process).  Rank r
of 2 owns envs [rN, (r+1)N).  rsl_rl's recurrent mini-batches are contiguous env slices
of each rank's shard, so mini-batch i of the two-rank run covers [rank 0's slice i,
rank 1's slice i].  The one-rank run over both shards therefore takes the 2N envs in that
interleaved order: its mini-batch i is exactly the union of the ranks' mini-batches i, and
(with equal slice sizes) the mean gradient, the mean KL and the global advantage
normalisation of the two-rank run are the one-rank run's.
"""
import os

import torch

T, N, O, P, A, H = 24, 512, 41, 44, 10, 64  # H1 shapes (h1_config.py:103-118), N envs per rank
EPOCHS, MINI_BATCHES = 2, 2


def rollout(num_envs, seed=5):
    """[T, num_envs, .] rollout + saved LSTM states (zero after a done) on the host."""
    g = torch.Generator().manual_seed(seed)
    r = dict(obs=torch.randn(T, num_envs, O, generator=g), cobs=torch.randn(T, num_envs, P, generator=g))
    mu = 0.3 * torch.randn(T, num_envs, A, generator=g)
    sigma = 0.8 * (1 + 0.1 * torch.rand(T, num_envs, A, generator=g))
    act = mu + sigma * torch.randn(T, num_envs, A, generator=g)
    r.update(mu=mu, sigma=sigma, actions=act,
             logp=torch.distributions.Normal(mu, sigma).log_prob(act).sum(-1, keepdim=True),
             values=0.5 * torch.randn(T, num_envs, 1, generator=g),
             rewards=0.2 * torch.randn(T, num_envs, 1, generator=g))
    dones = torch.rand(T, num_envs, 1, generator=g) < 0.04
    r["dones"] = dones
    hs = []
    for _ in range(2):
        s = 0.5 * torch.randn(T, 1, num_envs, H, generator=g)
        s[1:] *= (~dones[:-1, :, 0]).float().view(T - 1, 1, num_envs, 1)
        hs.append(s)
    r["hid"] = hs
    r["last_cobs"] = torch.randn(num_envs, P, generator=g)
    return r


def interleaved(world=2):
    """Env order of the one-rank run whose mini-batch i = the ranks' mini-batches i."""
    mb = N // MINI_BATCHES
    return torch.cat([torch.arange(r * N + i * mb, r * N + (i + 1) * mb)
                      for i in range(MINI_BATCHES) for r in range(world)])


def run(envs, device):
    """compute_returns + one update (EPOCHS x MINI_BATCHES, adaptive LR) over the envs
    `envs` (an index tensor into the 2N-env rollout); returns flat params, lr, losses."""
    from rsl_rl.algorithms import PPO
    from rsl_rl.modules import ActorCriticRecurrent
    torch.manual_seed(0)
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1, init_noise_std=0.8).to(device)
    alg = PPO(ac, num_learning_epochs=EPOCHS, num_mini_batches=MINI_BATCHES, learning_rate=1e-3,
              schedule="adaptive", desired_kl=0.01, gamma=0.99, lam=0.95, entropy_coef=0.01, device=device)
    alg.use_graph = False
    assert alg._dense_recurrent
    n = len(envs)
    alg.init_storage(n, T, [O], [P], [A])
    r = rollout(2 * N)
    st = alg.storage
    for name, key in (("observations", "obs"), ("privileged_observations", "cobs"), ("mu", "mu"),
                      ("sigma", "sigma"), ("actions", "actions"), ("actions_log_prob", "logp"),
                      ("values", "values"), ("rewards", "rewards")):
        getattr(st, name).copy_(r[key][:, envs])
    st.dones.copy_(r["dones"][:, envs].to(st.dones.dtype))
    st.saved_hidden_states_a = [h[:, :, envs].to(device).contiguous() for h in r["hid"]]
    st.saved_hidden_states_c = [(0.7 * h[:, :, envs]).to(device).contiguous() for h in r["hid"]]
    st.step = T
    alg.compute_returns(r["last_cobs"][envs].to(device))
    losses = alg.update()
    flat = torch.cat([p.detach().reshape(-1) for p in ac.parameters()]).cpu()
    return flat, alg.learning_rate, losses


def initial_params():
    from rsl_rl.modules import ActorCriticRecurrent
    torch.manual_seed(0)
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1, init_noise_std=0.8)
    return torch.cat([p.detach().reshape(-1) for p in ac.parameters()])


def worker(rank, world, port, device, q):
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(here, "..", "unitree-rl-gym_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if device.startswith("cuda"):
        torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        flat, lr, losses = run(torch.arange(rank * N, (rank + 1) * N), device)
        q.put((rank, flat.numpy(), lr, losses, None))
    except Exception:  # report, do not hang the parent
        import traceback
        q.put((rank, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def two_ranks(device, port):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, device, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[4] is None, r[4]
    return res
