"""Recurrent PPO update at H1 scale (8192 envs, T = 24, obs 41 / priv 44, 10 actions, LSTM 64,
MLP heads [32]; 5 epochs x 4 mini-batches): wall time of the update (eager and captured) and,
eager, a per-phase split of one optimizer step bracketed by HIP events.

usage: python tools/probes/recurrent_update_time.py [--trace]   (--trace: 2 eager updates only,
for a rocprofv3 kernel trace)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCriticRecurrent  # noqa: E402

T, N, O, P, A, H = 24, 8192, 41, 44, 10, 64


def fill(alg, seed=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    st = alg.storage
    st.observations.copy_(torch.randn(st.observations.shape, device="cuda", generator=g))
    st.privileged_observations.copy_(torch.randn(st.privileged_observations.shape, device="cuda", generator=g))
    mu = 0.3 * torch.randn(T, N, A, device="cuda", generator=g)
    sigma = 0.8 * (1 + 0.1 * torch.rand(T, N, A, device="cuda", generator=g))
    act = mu + sigma * torch.randn(T, N, A, device="cuda", generator=g)
    st.mu.copy_(mu)
    st.sigma.copy_(sigma)
    st.actions.copy_(act)
    st.actions_log_prob.copy_(torch.distributions.Normal(mu, sigma).log_prob(act).sum(-1, keepdim=True))
    st.values.copy_(0.5 * torch.randn(T, N, 1, device="cuda", generator=g))
    st.rewards.copy_(0.2 * torch.randn(T, N, 1, device="cuda", generator=g))
    dones = torch.rand(T, N, 1, device="cuda", generator=g) < 0.04
    st.dones.copy_(dones.to(st.dones.dtype))
    hs = []
    for _ in range(2):
        s = 0.5 * torch.randn(T, 1, N, H, device="cuda", generator=g)
        s[1:] *= (~dones[:-1, :, 0]).float().view(T - 1, 1, N, 1)
        hs.append(s)
    st.saved_hidden_states_a = hs
    st.saved_hidden_states_c = [0.7 * s for s in hs]
    st.step = T
    return torch.randn(N, P, device="cuda", generator=g)


def main():
    trace = "--trace" in sys.argv
    torch.manual_seed(0)
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1, init_noise_std=0.8).cuda()
    alg = PPO(ac, device="cuda", num_learning_epochs=5, num_mini_batches=4, learning_rate=1e-3,
              schedule="adaptive", entropy_coef=0.01)
    alg.init_storage(N, T, [O], [P], [A])
    last = fill(alg)
    alg.compute_returns(last)
    if trace:
        alg.use_graph = False
        for _ in range(2):
            alg.storage.step = T
            alg.update()
        torch.cuda.synchronize()
        return
    for mode in ("eager", "graph"):
        alg.use_graph = mode == "graph"
        for _ in range(2):
            alg.storage.step = T
            alg.update()
        torch.cuda.synchronize()
        R = 5
        t0 = time.time()
        for _ in range(R):
            alg.storage.step = T
            alg.update()
        torch.cuda.synchronize()
        print(f"{mode}: {(time.time() - t0) / R * 1e3:.2f} ms per update (20 optimizer steps)", flush=True)


if __name__ == "__main__":
    main()
