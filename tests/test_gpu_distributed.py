"""Data-parallel PPO on the fused GPU path (FusedPPOStep + the GAE kernels), two ranks.

Both ranks run on cuda:0 (one GPU per box here) with the gloo backend on CUDA tensors,
no graph capture; on an 8-GPU node the same code runs one rank per GPU over RCCL (bench.py
--gpus N).  Checked: (a) after an update the ranks hold bit-identical parameters; (b) two
ranks of N envs == one rank of the same 2N envs (global advantage normalisation through
the moments all-reduce, the mean gradient through the flat-bucket all-reduce, the global
KL for the adaptive learning rate), within the bf16 GEMMs' reduction-order tolerance.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

N, T, O, A = 512, 8, 48, 12
HID = [512, 256, 128]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rollout(num_envs, seed=3):
    """A synthetic rollout [T, num_envs, .] on the host (identical in every process)."""
    g = torch.Generator().manual_seed(seed)
    obs = torch.randn(T + 1, num_envs, O, generator=g)
    mu = 0.3 * torch.randn(T, num_envs, A, generator=g)
    sigma = torch.full((T, num_envs, A), 1.0) * (1 + 0.1 * torch.rand(T, num_envs, A, generator=g))
    act = mu + sigma * torch.randn(T, num_envs, A, generator=g)
    logp = torch.distributions.Normal(mu, sigma).log_prob(act).sum(-1, keepdim=True)
    return dict(obs=obs, mu=mu, sigma=sigma, actions=act, logp=logp,
                values=0.5 * torch.randn(T, num_envs, 1, generator=g),
                rewards=0.2 * torch.randn(T, num_envs, 1, generator=g),
                dones=(torch.rand(T, num_envs, 1, generator=g) < 0.05).to(torch.uint8))


def _run(envs):
    """One PPO update (compute_returns + 1 epoch x 1 mini-batch) on the fused path over
    the given env slice of the shared rollout; returns flat params, advantages, lr, losses."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(here, "..", "unitree-rl-gym_amd"), here]
    from rsl_rl.algorithms import PPO
    from rsl_rl.modules import ActorCritic
    torch.manual_seed(0)
    ac = ActorCritic(O, O, A, HID, HID, mixed_precision=True).cuda()
    alg = PPO(ac, num_learning_epochs=1, num_mini_batches=1, learning_rate=1e-3, schedule="adaptive",
              desired_kl=0.01, device="cuda")
    alg.use_graph = False
    n = envs.stop - envs.start
    alg.init_storage(n, T, [O], [None], [A])
    assert alg._fused is not None, "fused PPO step not active"
    r = _rollout(2 * N)
    st = alg.storage
    st.observations.copy_(r["obs"][:T, envs])
    st.actions.copy_(r["actions"][:, envs])
    st.mu.copy_(r["mu"][:, envs])
    st.sigma.copy_(r["sigma"][:, envs])
    st.actions_log_prob.copy_(r["logp"][:, envs])
    st.values.copy_(r["values"][:, envs])
    st.rewards.copy_(r["rewards"][:, envs])
    st.dones.copy_(r["dones"][:, envs].to(st.dones.dtype))
    st.step = T
    alg.compute_returns(r["obs"][T, envs].cuda())
    adv = st.advantages.detach().clone()
    torch.manual_seed(7)
    losses = alg.update()
    flat = torch.cat([p.detach().reshape(-1) for p in ac.parameters()]).cpu()
    return flat, adv.cpu(), alg.learning_rate, losses


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        flat, adv, lr, losses = _run(slice(rank * N, (rank + 1) * N))
        q.put((rank, flat.numpy(), adv.numpy(), lr, losses, None))
    except Exception as e:  # report, do not hang the parent
        import traceback
        q.put((rank, None, None, None, None, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_two_rank_fused_update_equals_one_rank_of_both_shards():
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[5] is None, r[5]
    # (a) identical parameters on every rank after the update
    assert np.array_equal(res[0][1], res[1][1])
    assert res[0][3] == res[1][3]
    # (b) == one rank over both shards
    flat1, adv1, lr1, losses1 = _run(slice(0, 2 * N))
    flat1 = flat1.numpy()
    adv1 = adv1.numpy()
    adv2 = np.concatenate([res[0][2], res[1][2]], axis=1)  # [T, N, 1] per rank -> [T, 2N, 1]
    np.testing.assert_allclose(adv2, adv1, rtol=1e-5, atol=1e-5)  # global advantage normalisation
    assert lr1 == pytest.approx(res[0][3], rel=1e-6)  # same KL decision
    np.testing.assert_allclose(res[0][4], losses1, rtol=2e-2, atol=2e-3)
    torch.manual_seed(0)
    from rsl_rl.modules import ActorCritic
    p0 = torch.cat([p.detach().reshape(-1) for p in ActorCritic(O, O, A, HID, HID).parameters()]).numpy()
    d1, d2 = flat1 - p0, res[0][1] - p0
    lr = 1e-3
    assert np.abs(d1).max() > 0
    bad = (np.abs(d1 - d2) > 0.2 * lr).mean()
    assert bad < 0.02, bad
    assert np.abs(d1 - d2).max() <= 4 * lr


_CAPTURE_PROBE = r"""
import os, sys
import torch
import torch.distributed as dist
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
x = torch.ones(4096, device="cuda")
dist.all_reduce(x)  # communicator set up outside the capture, as the first eager update does
torch.cuda.synchronize()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    x.mul_(3.0)
    dist.all_reduce(x)
torch.cuda.current_stream().wait_stream(s)
for _ in range(2):
    g.replay()
torch.cuda.synchronize()
assert float(x[0]) == 9.0 and bool((x == 9.0).all()), float(x[0])
dist.destroy_process_group()
print("captured all-reduce OK")
"""


def test_rccl_all_reduce_replays_inside_a_captured_graph():
    """The data-parallel update captures its gradient all-reduce (RCCL, backend "nccl") in
    the update graph.  The box has one GPU, so this checks the capture mechanics with one
    rank: an all-reduce recorded in a HIP graph replays (x *= 3, all-reduce, twice: 9)."""
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", _CAPTURE_PROBE], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "captured all-reduce OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_two_rank_recurrent_update_equals_one_rank_of_both_shards():
    """BASELINE configs[3]/[4] (H1 / H1_2 x 8 GPUs train ActorCriticRecurrent): two ranks of
    the dense recurrent update on the GPU (LSTM sequence kernels, fused PPO loss, GAE with the
    moments all-reduce; gloo on CUDA tensors, both ranks on cuda:0, no capture) at H1 shapes.
    One all-reduce per optimizer step carries the gradient bucket and the mini-batch KL.
    The ranks end bit-identical, and 2 x N envs == one rank of the same 2N envs (interleaved
    so its mini-batches are the ranks' unions) within the recurrent update's tolerance."""
    import dp_recurrent as dr
    res = dr.two_ranks("cuda", _free_port())
    assert np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]
    flat1, lr1, losses1 = dr.run(dr.interleaved(), "cuda")
    assert lr1 == pytest.approx(res[0][2], rel=1e-6)
    # each rank logs its own mini-batch means; their average is the union's mean
    np.testing.assert_allclose(0.5 * (np.array(res[0][3]) + np.array(res[1][3])), losses1, rtol=1e-3, atol=1e-5)
    p0 = dr.initial_params().numpy()
    d1, d2 = flat1.numpy() - p0, res[0][1] - p0
    lr = 1e-3
    assert np.abs(d1).max() > 0
    bad = (np.abs(d1 - d2) > 0.1 * lr).mean()
    assert bad < 0.02, bad
    assert np.abs(d1 - d2).max() <= 2 * dr.EPOCHS * dr.MINI_BATCHES * 1.5 * lr
