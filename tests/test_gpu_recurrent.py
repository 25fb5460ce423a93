"""The recurrent (LSTM) policy leg of BASELINE configs[2..4] (G1 / H1 / H1_2 train
ActorCriticRecurrent, LSTM 64): the HIP sequence kernels (csrc/lstm_seq.hip) against torch,
one recurrent PPO update at H1_2 scale against the same update in fp32 on the CPU (rsl_rl's
padded-trajectory form), and the captured rollout/update graphs against eager."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCriticRecurrent  # noqa: E402
from rsl_rl.modules import lstm_seq  # noqa: E402


@pytest.mark.parametrize("H,I", [(32, 47), (64, 47), (128, 47), (64, 17), (64, 64), (64, 80)])
def test_lstm_kernels_match_torch(H, I):
    """Forward outputs and the four parameter gradients of the dense LSTM (resets inside
    the sequence, a carried initial state) vs the same recurrence in torch fp32 ops.  I <= 64:
    the input projection inside the sequence kernel (pmlp_lstm_fwd_x); I = 80: a GEMM
    beforehand (pmlp_lstm_fwd)."""
    torch.manual_seed(H + I)
    T, B = 24, 1000
    rnn = torch.nn.LSTM(I, H).cuda()
    x = torch.randn(T, B, I, device="cuda")
    h0 = 0.5 * torch.randn(1, B, H, device="cuda")
    c0 = 0.5 * torch.randn(1, B, H, device="cuda")
    reset = (torch.rand(T, B, device="cuda") < 0.1).to(torch.uint8)
    reset[0] = 0
    y = lstm_seq.lstm_dense(rnn, x, h0, c0, reset, mfma=False)
    y_ref = lstm_seq.lstm_dense_reference(rnn, x, h0, c0, reset)
    torch.testing.assert_close(y, y_ref, rtol=1e-5, atol=2e-6)
    g = torch.randn_like(y)
    params = [rnn.weight_ih_l0, rnn.weight_hh_l0, rnn.bias_ih_l0, rnn.bias_hh_l0]
    gk = torch.autograd.grad(y, params, g)
    gr = torch.autograd.grad(y_ref, params, g)
    for name, a, b in zip(("w_ih", "w_hh", "b_ih", "b_hh"), gk, gr):
        rel = float((a - b).norm() / b.norm())
        assert rel < 1e-5, (name, rel)
    # without resets and from zeros, the reference statement is nn.LSTM itself
    y0 = lstm_seq.lstm_dense(rnn, x, None, None, None, mfma=False)
    torch.testing.assert_close(y0, rnn(x)[0], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("I", [41, 47, 64, 17])
def test_lstm_mfma_kernels_match_torch_to_bf16(I):
    """The update's matrix-core LSTM (pmlp_lstm_fwd_mfma / _bwd_mfma: split-bf16 operands,
    hi.hi + hi.lo + lo.hi products, fp32 accumulation and state) vs the same recurrence in
    torch fp32 ops over 24 steps with resets inside and a carried initial state: h within
    1e-4 absolute (h in [-1, 1]), the weight gradients within 1e-3 relative (norm); the
    weight-gradient operand [x | h_prev | 1] is the fp32 state."""
    torch.manual_seed(I)
    T, B, H = 24, 1000, 64
    rnn = torch.nn.LSTM(I, H).cuda()
    x = torch.randn(T, B, I, device="cuda")
    h0 = 0.5 * torch.randn(1, B, H, device="cuda")
    c0 = 0.5 * torch.randn(1, B, H, device="cuda")
    reset = (torch.rand(T, B, device="cuda") < 0.1).to(torch.uint8)
    reset[0, :7] = 1
    y = lstm_seq.lstm_dense(rnn, x, h0, c0, reset, mfma=True)
    y_ref = lstm_seq.lstm_dense_reference(rnn, x, h0, c0, reset)
    err = float((y - y_ref).abs().max())
    print("mfma lstm max |dh|", err)
    assert err < 1e-4
    assert float((y - y_ref).norm() / y_ref.norm()) < 1e-4
    g = torch.randn_like(y)
    params = [rnn.weight_ih_l0, rnn.weight_hh_l0, rnn.bias_ih_l0, rnn.bias_hh_l0]
    gk = torch.autograd.grad(y, params, g)
    gr = torch.autograd.grad(y_ref, params, g)
    for name, a, b in zip(("w_ih", "w_hh", "b_ih", "b_hh"), gk, gr):
        rel = float((a - b).norm() / b.norm())
        print("mfma lstm grad", name, rel)
        assert rel < 1e-3, (name, rel)


def test_lstm_fused_input_writes_the_weight_gradient_operand():
    """pmlp_lstm_fwd_x's xh = [x | h_prev | 1]: h_prev is the state each step starts from
    (h0 at t = 0, zero after a reset, else the previous output)."""
    torch.manual_seed(1)
    T, B, I, H = 6, 37, 41, 64
    rnn = torch.nn.LSTM(I, H).cuda()
    x = torch.randn(T, B, I, device="cuda")
    h0 = torch.randn(B, H, device="cuda")
    c0 = torch.randn(B, H, device="cuda")
    reset = (torch.rand(T, B, device="cuda") < 0.3).to(torch.uint8)
    h_out = torch.empty(T, B, H, device="cuda")
    xh = torch.full((T, B, I + H + 1), float("nan"), device="cuda")
    p = lstm_seq.mm._p
    lib = lstm_seq._lib()
    w = [t.detach().contiguous() for t in (rnn.weight_ih_l0, rnn.bias_ih_l0, rnn.bias_hh_l0, rnn.weight_hh_l0)]
    assert lib.pmlp_lstm_fwd_x(T, B, H, I, p(x), p(w[0]), p(w[1]), p(w[2]), p(w[3]), p(h0), p(c0), p(reset),
                               p(h_out), None, None, None, None, p(xh), lstm_seq.mm._stream()) == 0
    torch.cuda.synchronize()
    hp = torch.cat([h0.unsqueeze(0), h_out[:-1]]) * (reset == 0).float().unsqueeze(-1)
    assert torch.equal(xh[..., :I], x)
    assert torch.equal(xh[..., I:I + H], hp)
    assert bool((xh[..., I + H] == 1).all())


def test_lstm_rollout_step_in_place_matches_nn_lstm():
    torch.manual_seed(0)
    B, I, H = 8192, 47, 64
    rnn = torch.nn.LSTM(I, H).cuda()
    h = 0.3 * torch.randn(1, B, H, device="cuda")
    c = 0.3 * torch.randn(1, B, H, device="cuda")
    x = torch.randn(B, I, device="cuda")
    out_ref, (h_ref, c_ref) = rnn(x.unsqueeze(0), (h.clone(), c.clone()))
    ptr = h.data_ptr()
    out = lstm_seq.lstm_step_(rnn, x, h, c)
    assert out.data_ptr() == ptr  # in place: static state buffers
    torch.testing.assert_close(h, h_ref, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(c, c_ref, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(out, out_ref, rtol=1e-5, atol=2e-6)


def _synthetic_storage(alg, T, N, O, P, A, H, seed):
    """A rollout with dones and the saved hidden states of a real recurrent rollout: the
    state at t = 0 is carried (nonzero); after a done it is zero."""
    g = torch.Generator().manual_seed(seed)
    st = alg.storage
    st.observations.copy_(torch.randn(T, N, O, generator=g))
    st.privileged_observations.copy_(torch.randn(T, N, P, generator=g))
    mu = 0.3 * torch.randn(T, N, A, generator=g)
    sigma = 0.8 * (1 + 0.1 * torch.rand(T, N, A, generator=g))
    act = mu + sigma * torch.randn(T, N, A, generator=g)
    st.mu.copy_(mu)
    st.sigma.copy_(sigma)
    st.actions.copy_(act)
    st.actions_log_prob.copy_(torch.distributions.Normal(mu, sigma).log_prob(act).sum(-1, keepdim=True))
    st.values.copy_(0.5 * torch.randn(T, N, 1, generator=g))
    st.rewards.copy_(0.2 * torch.randn(T, N, 1, generator=g))
    dones = (torch.rand(T, N, 1, generator=g) < 0.04)
    st.dones.copy_(dones.to(st.dones.dtype))
    hs = []
    for _ in range(2):  # (h, c)
        s = 0.5 * torch.randn(T, 1, N, H, generator=g)
        s[1:] *= (~dones[:-1, :, 0]).float().view(T - 1, 1, N, 1)
        hs.append(s)
    dev = st.observations.device
    st.saved_hidden_states_a = [s.to(dev) for s in hs]
    st.saved_hidden_states_c = [(0.7 * s).to(dev) for s in hs]
    st.step = T
    return torch.randn(N, P, generator=g)


def test_recurrent_ppo_update_matches_fp32_cpu_update():
    """One PPO update (5 epochs x 4 mini-batches, adaptive LR) of the H1_2 recurrent policy at
    BASELINE scale (obs 47, priv 50, 8192 envs, T = 24, LSTM 64, MLP [32]) on the GPU (dense
    form, LSTM kernels, GAE kernel) vs the same update on the CPU in fp32 with rsl_rl's padded
    trajectories and torch's LSTM."""
    T, N, O, P, A, H = 24, 8192, 47, 50, 12, 64
    torch.manual_seed(0)
    kw = dict(actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm", rnn_hidden_size=H,
              rnn_num_layers=1, init_noise_std=0.8)
    ac_cpu = ActorCriticRecurrent(O, P, A, **kw)
    ac_gpu = copy.deepcopy(ac_cpu).cuda()
    akw = dict(num_learning_epochs=5, num_mini_batches=4, learning_rate=1e-3, schedule="adaptive", gamma=0.99,
               lam=0.95, entropy_coef=0.01)
    cpu = PPO(ac_cpu, device="cpu", **akw)
    cpu._dense_recurrent = False  # rsl_rl's own padded-trajectory generator
    gpu = PPO(ac_gpu, device="cuda", **akw)
    assert gpu._dense_recurrent and gpu.use_graph
    for alg in (cpu, gpu):
        alg.init_storage(N, T, [O], [P], [A])
    last = _synthetic_storage(cpu, T, N, O, P, A, H, seed=1)
    _synthetic_storage(gpu, T, N, O, P, A, H, seed=1)
    cpu.compute_returns(last)
    gpu.compute_returns(last.cuda())
    torch.testing.assert_close(gpu.storage.advantages.cpu(), cpu.storage.advantages, rtol=1e-4, atol=1e-4)
    p0 = [p.detach().clone() for p in ac_cpu.parameters()]
    l_cpu = cpu.update()
    l_gpu = gpu.update()  # eager (first call)
    np.testing.assert_allclose(l_gpu, l_cpu, rtol=1e-3, atol=1e-5)
    assert gpu.learning_rate == pytest.approx(cpu.learning_rate, rel=1e-6)
    lr = 1e-3
    for (name, a), b, c in zip(ac_cpu.named_parameters(), ac_gpu.parameters(), p0):
        da, db = a.detach() - c, b.detach().cpu() - c
        assert da.abs().max() > 0, name
        # Adam turns a sign flip of a ~0 gradient into a ~lr move: a few entries may differ
        # (at most 2 %, or one entry of a small tensor such as the critic's 32 output weights)
        nbad = int(((da - db).abs() > 0.1 * lr).sum())
        assert nbad <= max(1, 0.02 * da.numel()), (name, nbad, da.numel())
        assert (da - db).abs().max() <= 2 * 20 * 1.5 * lr, name


def test_recurrent_update_graph_matches_eager():
    """The captured recurrent update (dense generator, LSTM kernels, capturable Adam) replays
    the eager update: same losses and parameters from the same starting point."""
    T, N, O, P, A, H = 24, 2048, 47, 50, 12, 64
    torch.manual_seed(0)
    kw = dict(actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm", rnn_hidden_size=H,
              rnn_num_layers=1, init_noise_std=0.8)
    ac = ActorCriticRecurrent(O, P, A, **kw).cuda()
    alg = PPO(ac, device="cuda", num_learning_epochs=2, num_mini_batches=4, learning_rate=3e-4, schedule="fixed")
    alg.init_storage(N, T, [O], [P], [A])
    last = _synthetic_storage(alg, T, N, O, P, A, H, seed=2).cuda()
    alg.compute_returns(last)
    alg.update()  # eager warm-up
    graph_of = lambda a: a._graph if a._rfused is None else a._rgraph  # noqa: E731
    assert graph_of(alg) is None
    saved = {k: v.clone() for k, v in alg.storage.__dict__.items() if torch.is_tensor(v) and not k.startswith("_")}
    params = list(ac.parameters())
    p0 = [p.detach().clone() for p in params]
    st0 = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in alg.optimizer.state[p].items()}
           for p in params}
    alg.storage.step = T
    g_loss = alg.update()  # captured + replayed
    assert graph_of(alg) is not None
    p_graph = [p.detach().clone() for p in params]
    with torch.no_grad():
        for p, v in zip(params, p0):
            p.copy_(v)
        for p in params:
            for k, v in alg.optimizer.state[p].items():
                if torch.is_tensor(v):
                    v.copy_(st0[id(p)][k])
        for k, v in saved.items():
            getattr(alg.storage, k).copy_(v)
    alg.storage.step = T
    alg.use_graph = False
    e_loss = alg.update()
    np.testing.assert_allclose(g_loss, e_loss, rtol=1e-5, atol=1e-7)
    for a, b in zip(params, p_graph):
        assert (a.detach() - b).abs().max() <= 8 * 3e-4


def test_recurrent_rollout_graph_matches_eager(tmp_path):
    """OnPolicyRunner on H1 (recurrent policy): the captured collection loop (LSTM state
    stepped in place, masked resets) replays the eager loop's rollouts."""
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry
    from legged_gym.utils import get_args
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    out = {}
    for graph in (False, True):
        args = get_args(["--task", "h1", "--num_envs", "512", "--headless"])
        env_cfg, train_cfg = task_registry.get_cfgs("h1")
        env_cfg = copy.deepcopy(env_cfg)
        env_cfg.env.episode_length_s = 0.5  # resets inside every rollout
        env, _ = task_registry.make_env(name="h1", args=args, env_cfg=env_cfg)
        cfg = class_to_dict(train_cfg)
        cfg["runner"]["rollout_graph"] = graph
        torch.manual_seed(0)
        torch.cuda.manual_seed(0)
        runner = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
        runner.alg.use_graph = False  # compare the rollouts, not the update paths
        runner.learn(3, init_at_random_ep_len=True)
        torch.cuda.synchronize()
        st = runner.alg.storage
        out[graph] = dict(root=env.root_states.clone(), st_obs=st.observations.clone(), st_act=st.actions.clone(),
                          st_rew=st.rewards.clone(), hid=st.saved_hidden_states_a[0].clone(),
                          mem=runner.alg.actor_critic.memory_a.hidden_states[0].clone(),
                          params=[p.detach().clone() for p in runner.alg.actor_critic.parameters()],
                          captured=runner._rollout_graph is not None)
        env.close()
    e, g = out[False], out[True]
    assert g["captured"] and not e["captured"]
    for k in ("root", "st_obs", "st_act", "st_rew", "hid", "mem"):
        assert torch.equal(e[k], g[k]), k
    for a, b in zip(e["params"], g["params"]):
        assert torch.equal(a, b)


def test_recurrent_rollout_saves_the_pre_step_state_from_the_kernel():
    """RecurrentRollout: the storage slot of step t holds the memory state the step started
    from (written by the LSTM step kernel itself), as RolloutStorage._save_hidden_states
    would copy it; step 0 of the first rollout starts from zeros."""
    torch.manual_seed(3)
    N, T, O, P, A, H = 256, 4, 47, 50, 12, 64
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1).cuda()
    alg = PPO(ac, device="cuda")
    alg.init_storage(N, T, [O], [P], [A])
    assert alg._rollout is not None
    st = alg.storage
    for t in range(T):
        obs, cobs = torch.randn(N, O, device="cuda"), torch.randn(N, P, device="cuda")
        prev = [None if s is None else s.clone() for s in (ac.memory_a.hidden_states or (None, None))] + \
               [None if s is None else s.clone() for s in (ac.memory_c.hidden_states or (None, None))]
        rew, done = torch.randn(N, device="cuda"), torch.rand(N, device="cuda") < 0.2
        tout = torch.rand(N, device="cuda") < 0.5
        with torch.inference_mode():
            alg.act(obs, cobs)
            alg.process_env_step(rew, done, {"time_outs": tout})
        alg.flush_rollout()
        # process_env_step's storage rows (rsl_rl ppo.py: reward bootstrapped on time-outs)
        want = rew + alg.gamma * st.values[t].squeeze(1) * tout.float()
        torch.testing.assert_close(st.rewards[t].squeeze(1), want, rtol=1e-6, atol=1e-6)
        assert torch.equal(st.dones[t].view(-1).bool(), done)
        got = [st.saved_hidden_states_a[0][t], st.saved_hidden_states_a[1][t], st.saved_hidden_states_c[0][t],
               st.saved_hidden_states_c[1][t]]
        for g, p in zip(got, prev):
            if p is None:
                assert bool((g == 0).all())
            else:
                assert torch.equal(g, p)


@pytest.mark.parametrize("robot", ["g1", "h1", "h1_2"])
def test_hip_lstm_matches_pretrained_policy_golden(robot):
    """The reference's own pretrained recurrent policies (deploy/pre_train/<robot>/motion.pt,
    extracted to tests/golden/lstm_policy_<robot>.npz: weights + the 20-step outputs from a
    fresh memory and again after reset_memory) through the HIP LSTM kernels:
    (a) the in-place rollout step (Memory.step_ -> pmlp_lstm_step, what act_inference and the
        captured rollout run), with a reset of the memory rows before the second sequence;
    (b) the dense sequence kernel of the update (lstm_dense), with the reset mask.
    The golden sequence sits in a few rows of a batch of random envs (the kernels index envs
    correctly) and must match at 1e-5 (helpers.py:163-189 PolicyExporterLSTM semantics)."""
    import os
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, f"lstm_policy_{robot}.npz"))
    n_in = g["w.memory.weight_ih_l0"].shape[1]
    n_act = g["w.actor.2.weight"].shape[0]
    ac = ActorCriticRecurrent(n_in, n_in + 3, n_act, actor_hidden_dims=[32], critic_hidden_dims=[32],
                              rnn_type="lstm", rnn_hidden_size=64, rnn_num_layers=1, init_noise_std=0.8)
    sd = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w.")}
    ac.actor.load_state_dict({k[len("actor."):]: v for k, v in sd.items() if k.startswith("actor.")})
    ac.memory_a.rnn.load_state_dict({k[len("memory."):]: v for k, v in sd.items() if k.startswith("memory.")})
    ac = ac.cuda().eval()
    xs = torch.from_numpy(g["inputs"]).cuda()  # [20, n_in]
    steps, B, rows = xs.shape[0], 1000, [0, 517, 999]
    torch.manual_seed(11)
    seq = torch.randn(steps + 5, B, n_in, device="cuda")
    for r in rows:
        seq[:steps, r] = xs
        seq[steps:, r] = xs[:5]
    reset = torch.zeros(steps + 5, B, dtype=torch.uint8, device="cuda")
    reset[steps, rows] = 1
    want = torch.from_numpy(np.concatenate([g["outputs"], g["outputs_after_reset"]])).cuda()
    # (a) rollout steps in place (act_inference: Memory.forward -> lstm_seq.lstm_step_)
    ac.memory_a.hidden_states = None
    got = []
    with torch.no_grad():
        for t in range(steps + 5):
            if t == steps:
                ac.memory_a.reset(reset[t].bool())
            got.append(ac.act_inference(seq[t]))
    got = torch.stack(got)
    assert lstm_seq.usable(ac.memory_a.rnn, seq[0])
    for r in rows:
        torch.testing.assert_close(got[:, r], want, rtol=1e-5, atol=1e-5)
    # (b) the dense sequence kernels (the update's forward), zero state at t = 0: the fp32
    # kernel at 1e-5, the matrix-core kernel (split-bf16 operands, ~2^-16 relative per
    # product) at 2e-4 on the action means
    for mfma, tol in ((False, 1e-5), (True, 2e-4)):
        with torch.no_grad():
            h = lstm_seq.lstm_dense(ac.memory_a.rnn, seq, None, None, reset, mfma=mfma)
            mu = ac.actor(h.reshape(-1, 64)).view(steps + 5, B, n_act)
        for r in rows:
            torch.testing.assert_close(mu[:, r], want, rtol=tol, atol=tol)


@pytest.mark.parametrize("M", [1000, 20003])
@pytest.mark.parametrize("H", [32, 64, 128])
def test_fused_recurrent_heads_match_torch(H, M):
    """pmlp_heads_forward / pmlp_heads_backward (the fused recurrent step's MLP heads, fp32) vs
    torch autograd of Sequential(Linear(H, 32), ELU, Linear(32, N1)) for the actor (N1 = 12)
    and the critic (N1 = 1) in one launch each, on row counts that are not a multiple of the
    64- or 128-row blocks (20,003: the forward's matrix-core form, from 16,384 rows); the
    per-block weight-gradient partials summed by pmlp_reduce_slabs."""
    from rsl_rl.modules import mfma_mlp as mm
    torch.manual_seed(H)
    N0 = 32
    nets = [torch.nn.Sequential(torch.nn.Linear(H, N0), torch.nn.ELU(), torch.nn.Linear(N0, n1)).cuda()
            for n1 in (12, 1)]
    hs = [torch.randn(M, H, device="cuda") for _ in range(2)]
    douts = [torch.randn(M, n.__getitem__(2).out_features, device="cuda") for n in nets]
    lib = mm.load()
    nblk = lib.pmlp_heads_blocks(M)
    bufs = []
    for n, net in enumerate(nets):
        n1 = net[2].out_features
        nh = N0 * H + N0 + n1 * N0 + n1
        bufs.append(dict(y0=torch.empty(M, N0, device="cuda"), out=torch.empty(M, n1, device="cuda"),
                         dh=torch.empty(M, H, device="cuda"), slab=torch.empty(nblk, nh, device="cuda"),
                         grad=torch.empty(nh, device="cuda"), nh=nh))
    P = mm._p
    jobs = (mm.HeadJob * 2)(*[mm.HeadJob(P(hs[n]), P(net[0].weight), P(net[0].bias), P(net[2].weight), P(net[2].bias),
                                         P(bufs[n]["y0"]), P(bufs[n]["out"]), P(douts[n]), P(bufs[n]["dh"]),
                                         P(bufs[n]["slab"]), N0, net[2].out_features) for n, net in enumerate(nets)])
    mm._ok(lib.pmlp_heads_forward(2, jobs, M, H, mm._stream()), "pmlp_heads_forward")
    mm._ok(lib.pmlp_heads_backward(2, jobs, M, H, mm._stream()), "pmlp_heads_backward")
    mm._reduce([(b["slab"], b["grad"], b["nh"], nblk) for b in bufs])
    for n, net in enumerate(nets):
        h = hs[n].clone().requires_grad_(True)
        y0 = torch.nn.functional.elu(net[0](h))
        out = net[2](y0)
        torch.testing.assert_close(bufs[n]["y0"], y0.detach(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(bufs[n]["out"], out.detach(), rtol=1e-5, atol=1e-5)
        params = [net[0].weight, net[0].bias, net[2].weight, net[2].bias]
        g = torch.autograd.grad(out, [h] + params, douts[n])
        torch.testing.assert_close(bufs[n]["dh"], g[0], rtol=1e-5, atol=1e-5)
        # the weight gradients are fp32 sums over the M rows, in another order than any fp32
        # reference's: against fp64, with an absolute tolerance growing as sqrt(M) (1e-4 at
        # M = 1000; measured 2.2e-4 against torch's fp32 GEMM at M = 20,003)
        net64 = copy.deepcopy(net).double()
        h64 = hs[n].double().requires_grad_(True)
        out64 = net64[2](torch.nn.functional.elu(net64[0](h64)))
        g64 = torch.autograd.grad(out64, [net64[0].weight, net64[0].bias, net64[2].weight, net64[2].bias],
                                  douts[n].double())
        want = torch.cat([t.reshape(-1) for t in g64]).float()
        torch.testing.assert_close(bufs[n]["grad"], want, rtol=1e-4, atol=1e-4 * max(1.0, M / 1000) ** 0.5)


@pytest.mark.parametrize("I", [41, 47, 17, 63])
def test_lstm_bwd_accumulates_the_weight_gradients(I):
    """pmlp_lstm_bwd_dw_mfma (the fused recurrent step's memory backward): the per-workgroup
    partials of dG^T [x | h_prev | 1], summed over the slab rows, are the weight gradients of
    torch autograd through the same recurrence (resets inside, a carried initial state; env
    count not a multiple of the 16-env workgroups), within 1e-4 relative (norm)."""
    from rsl_rl.modules import mfma_mlp as mm
    torch.manual_seed(I)
    T, B, H = 24, 1000, 64
    rnn = torch.nn.LSTM(I, H).cuda()
    x = torch.randn(T, B, I, device="cuda")
    h0 = 0.5 * torch.randn(B, H, device="cuda")
    c0 = 0.5 * torch.randn(B, H, device="cuda")
    reset = (torch.rand(T, B, device="cuda") < 0.1).to(torch.uint8)
    g = torch.randn(T, B, H, device="cuda")
    L, P, st = lstm_seq._lib(), mm._p, mm._stream()
    h_out, c_out = torch.empty(T, B, H, device="cuda"), torch.empty(T, B, H, device="cuda")
    gact, xh = torch.empty(T, B, 4 * H, device="cuda"), torch.empty(T, B, I + H + 1, device="cuda")
    w = [t.detach().contiguous() for t in (rnn.weight_ih_l0, rnn.bias_ih_l0, rnn.bias_hh_l0, rnn.weight_hh_l0)]
    lstm_seq._ok(L.pmlp_lstm_fwd_mfma(T, B, H, I, P(x), P(w[0]), P(w[1]), P(w[2]), P(w[3]), P(h0), P(c0), P(reset),
                                      P(h_out), P(c_out), P(gact), P(xh), st), "fwd")
    nblk = L.pmlp_lstm_bwd_dw_blocks(B)
    slab = torch.empty(nblk, 4 * H * (I + H + 1), device="cuda")
    lstm_seq._ok(L.pmlp_lstm_bwd_dw_mfma(T, B, H, I, P(w[3]), P(c0), P(reset), P(c_out), P(gact), P(g), P(xh),
                                         P(slab), st), "bwd_dw")
    tot = slab.sum(0)
    got = [tot[:4 * H * I].view(4 * H, I), tot[4 * H * I:4 * H * (I + H)].view(4 * H, H), tot[4 * H * (I + H):]]
    y_ref = lstm_seq.lstm_dense_reference(rnn, x, h0, c0, reset)
    want = torch.autograd.grad(y_ref, [rnn.weight_ih_l0, rnn.weight_hh_l0, rnn.bias_ih_l0], g)
    for name, a, b in zip(("w_ih", "w_hh", "b"), got, want):
        rel = float((a - b).norm() / b.norm())
        assert rel < 1e-4, (name, rel)


def test_recurrent_rollout_heads_kernel_matches_torch_heads():
    """RecurrentRollout runs both MLP heads in one pmlp_heads_forward launch: the stored action
    means and values equal the torch heads on the memories' new state within 1e-5."""
    torch.manual_seed(3)
    N, T, O, P, A, H = 1000, 4, 41, 44, 10, 64
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1, init_noise_std=0.8).cuda()
    alg = PPO(ac, device="cuda", num_learning_epochs=1, num_mini_batches=1)
    alg.init_storage(N, T, [O], [P], [A])
    assert alg._rollout is not None and alg._rollout.heads is not None
    obs, cobs = torch.randn(N, O, device="cuda"), torch.randn(N, P, device="cuda")
    with torch.inference_mode():
        alg.act(obs, cobs)
        ha, hc = ac.memory_a.hidden_states[0][0], ac.memory_c.hidden_states[0][0]
        mu, value = ac.actor(ha), ac.critic(hc)
    torch.testing.assert_close(alg.storage.mu[0], mu, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(alg.storage.values[0], value, rtol=1e-5, atol=1e-5)


def test_lstm_rollout_step_mfma_in_place_matches_nn_lstm():
    """pmlp_lstm_step_mfma (the recurrent rollout's memory step: the update's matrix-core
    arithmetic at T = 1): h, c updated in place and the pre-step state saved, vs one nn.LSTM
    step within the split-bf16 tolerance (2e-5), over three steps."""
    torch.manual_seed(5)
    B, I, H = 1000, 44, 64
    rnn = torch.nn.LSTM(I, H).cuda()
    h = 0.5 * torch.randn(1, B, H, device="cuda")
    c = 0.5 * torch.randn(1, B, H, device="cuda")
    hs, cs = torch.empty_like(h), torch.empty_like(c)
    for _ in range(3):
        x = torch.randn(B, I, device="cuda")
        h_ref, c_ref = h.clone(), c.clone()
        with torch.no_grad():
            y, (h_new, c_new) = rnn(x.unsqueeze(0), (h_ref, c_ref))
        out = lstm_seq.lstm_step_mfma_(rnn, x, h, c, save=(hs, cs))
        assert out.data_ptr() == h.data_ptr()
        assert torch.equal(hs, h_ref) and torch.equal(cs, c_ref)
        torch.testing.assert_close(h, h_new, rtol=2e-5, atol=2e-5)
        torch.testing.assert_close(c, c_new, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("done_dtype", [torch.bool, torch.int64])
def test_recurrent_rollout_draws_fresh_noise_every_step_and_iteration(done_dtype):
    """the recurrent rollout's Philox draw counter advances after every
    pmlp_act (in pmlp_store_step), so the standardised noise (a - mu) / sigma differs between
    consecutive steps and between iterations (storage cleared, same obs).  ADVICE r5: long
    dones (the reference's reset_buf dtype) take process_env_step's generic branch, which
    advances the counter itself."""
    torch.manual_seed(4)
    N, T, O, P, A, H = 256, 3, 47, 50, 12, 64
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1).cuda()
    alg = PPO(ac, device="cuda")
    alg.init_storage(N, T, [O], [P], [A])
    assert alg._rollout is not None
    st = alg.storage
    g = torch.Generator(device="cuda").manual_seed(1)
    obs, cobs = torch.randn(N, O, device="cuda", generator=g), torch.randn(N, P, device="cuda", generator=g)
    zs = []
    for it in range(2):
        for t in range(T):
            with torch.inference_mode():
                alg.act(obs, cobs)
                alg.process_env_step(torch.zeros(N, device="cuda"), torch.zeros(N, dtype=done_dtype, device="cuda"),
                                     {"time_outs": torch.zeros(N, dtype=torch.bool, device="cuda")})
            zs.append(((st.actions[t] - st.mu[t]) / st.sigma[t]).clone())
        alg.flush_rollout()
        st.clear()
    for i in range(len(zs)):
        for j in range(i):
            same = (zs[i] == zs[j]).float().mean().item()
            assert same < 0.01, (i, j, same)
    z = torch.stack(zs)
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 1.0) < 0.02


def test_recurrent_store_zeroes_the_done_envs_memories_as_reset():
    """The recurrent rollout's store launch zeroes the done envs' (h, c) of both memories
    itself (pmlp_store_step_reset): bitwise ActorCriticRecurrent.reset(dones) (masked_fill_
    with 0), the other envs' states untouched, and PPO.process_env_step then skips the
    torch statement."""
    torch.manual_seed(5)
    N, T, O, P, A, H = 256, 3, 47, 50, 12, 64
    ac = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=H, rnn_num_layers=1).cuda()
    alg = PPO(ac, device="cuda")
    alg.init_storage(N, T, [O], [P], [A])
    g = torch.Generator(device="cuda").manual_seed(2)
    obs, cobs = torch.randn(N, O, device="cuda", generator=g), torch.randn(N, P, device="cuda", generator=g)
    calls = []
    real_reset = ac.reset
    ac.reset = lambda dones=None: (calls.append(1), real_reset(dones))[1]
    for t in range(T):
        with torch.inference_mode():
            alg.act(obs, cobs)
            before = [h.clone() for m in (ac.memory_a, ac.memory_c) for h in m.hidden_states]
            assert all(bool((h != 0).any()) for h in before)
            dones = torch.rand(N, device="cuda", generator=g) < 0.2
            alg.process_env_step(torch.zeros(N, device="cuda"), dones,
                                 {"time_outs": torch.zeros(N, dtype=torch.bool, device="cuda")})
            after = [h for m in (ac.memory_a, ac.memory_c) for h in m.hidden_states]
        for b, a in zip(before, after):
            ref = b.masked_fill(dones.view(1, -1, 1), 0.0)
            assert torch.equal(a, ref)
    assert not calls  # the torch reset was not needed


def test_recurrent_heads_with_fused_sampling_are_bitwise_the_separate_launches():
    """pmlp_heads_forward_act (the actor's sampling and the storage rows in the heads' launch)
    against pmlp_heads_forward + pmlp_act: from identical policies, memories and noise keys,
    the actions and every storage row are bitwise the same over a few steps."""
    import copy
    torch.manual_seed(6)
    N, T, O, P, A, H = 512, 3, 47, 50, 12, 64
    ac0 = ActorCriticRecurrent(O, P, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                               rnn_hidden_size=H, rnn_num_layers=1).cuda()
    algs = []
    for fuse in (False, True):
        torch.manual_seed(11)  # the rollout's noise seed
        alg = PPO(copy.deepcopy(ac0), device="cuda")
        alg.init_storage(N, T, [O], [P], [A])
        assert alg._rollout is not None and alg._rollout.heads is not None
        alg._rollout.fuse_act = fuse
        algs.append(alg)
    assert algs[0]._rollout.seed == algs[1]._rollout.seed
    g = torch.Generator(device="cuda").manual_seed(3)
    for t in range(T):
        obs, cobs = torch.randn(N, O, device="cuda", generator=g), torch.randn(N, P, device="cuda", generator=g)
        dones = torch.rand(N, device="cuda", generator=g) < 0.1
        acts = []
        for alg in algs:
            with torch.inference_mode():
                acts.append(alg.act(obs, cobs).clone())
                alg.process_env_step(torch.ones(N, device="cuda"), dones,
                                     {"time_outs": torch.zeros(N, dtype=torch.bool, device="cuda")})
        assert torch.equal(acts[0], acts[1])
    sa, sb = algs[0].storage, algs[1].storage
    for k in ("actions", "actions_log_prob", "mu", "sigma", "values", "observations", "privileged_observations",
              "rewards", "dones"):
        assert torch.equal(getattr(sa, k), getattr(sb, k)), k


def test_recurrent_heads_matrix_core_form_is_bitwise_the_valu_form():
    """The heads' products on the matrix cores (default) against the VALU form
    (PMLP_HEADS_MFMA=0, read once per process: two probe processes), y0, out, dh and the
    weight-gradient slabs digested, on 20,003 rows (the forward's matrix-core form, ragged
    last tiles).  Each f32 MFMA chain keeps the VALU form's fma order (lstm_seq.hip)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    digests = []
    for flag in ("1", "0"):
        env = dict(os.environ, PMLP_HEADS_MFMA=flag)
        out = subprocess.run([sys.executable, os.path.join(root, "tools", "probes", "heads_time.py"), "20003"],
                             env=env, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr[-2000:]
        digests.append(out.stdout.strip().rsplit("outputs ", 1)[1])
    assert digests[0] == digests[1]
