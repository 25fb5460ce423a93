"""The fused PPO optimizer step (rsl_rl/algorithms/fused_step.py: gathered bf16
MFMA forward/backward, fused loss, flat clip_grad_norm_ + Adam, GAE kernel)
against the reference's torch statement of the same update (fp32 autograd,
nn.utils.clip_grad_norm_, torch.optim.Adam, RolloutStorage.compute_returns)."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.algorithms import fused_step  # noqa: E402
from rsl_rl.modules import ActorCritic, mfma_mlp  # noqa: E402
from rsl_rl.storage import RolloutStorage  # noqa: E402


def _fill_storage(alg, T, N, O, A, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    st = alg.storage
    ro, alg._rollout = alg._rollout, None  # the reference act()/process_env_step path (custom actions)
    with torch.inference_mode():
        for _ in range(T):
            obs = torch.randn(N, O, device="cuda", generator=g)
            alg.act(obs, obs)
            alg.transition.actions = alg.transition.action_mean + 0.3 * torch.randn(N, A, device="cuda", generator=g)
            alg.transition.actions_log_prob = alg.actor_critic.get_actions_log_prob(alg.transition.actions).detach()
            rew = 0.2 * torch.randn(N, device="cuda", generator=g)
            done = torch.rand(N, device="cuda", generator=g) < 0.05
            alg.process_env_step(rew, done, {"time_outs": done & (torch.rand(N, device="cuda", generator=g) < 0.5)})
        alg.compute_returns(torch.randn(N, O, device="cuda", generator=g))
    alg._rollout = ro
    return {k: v.clone() for k, v in st.__dict__.items() if torch.is_tensor(v) and not k.startswith("_")}


@pytest.mark.parametrize("schedule", ["fixed", "adaptive"])
def test_fused_step_matches_fp32_autograd_update(schedule):
    """One update (1 epoch x 2 mini-batches) from identical weights and rollout:
    losses, learning rate and every parameter after the two Adam steps agree with
    the fp32 torch update within bf16 GEMM rounding."""
    torch.manual_seed(0)
    N, T, O, A = 1024, 8, 48, 12
    ac32 = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128], mixed_precision=False).cuda()
    acbf = copy.deepcopy(ac32)
    acbf.mixed_precision = True
    kw = dict(num_learning_epochs=1, num_mini_batches=2, learning_rate=1e-3, schedule=schedule, device="cuda")
    ref = PPO(ac32, fused_loss=False, **kw)
    ref.use_graph = False
    fus = PPO(acbf, **kw)
    for alg in (ref, fus):
        alg.init_storage(N, T, [O], [None], [A])
    assert fus._fused is not None and ref._fused is None
    data = _fill_storage(ref, T, N, O, A, seed=1)
    for k, v in data.items():  # identical rollout for both
        getattr(fus.storage, k).copy_(v)
    fus.storage.step = T
    p0 = [p.detach().clone() for p in ref.actor_critic.parameters()]
    torch.manual_seed(7)
    l_ref = ref.update()
    torch.manual_seed(7)
    l_fus = fus.update()
    np.testing.assert_allclose(l_fus, l_ref, rtol=2e-2, atol=2e-3)
    assert fus.learning_rate == pytest.approx(ref.learning_rate, rel=1e-6)
    lr = 1e-3
    for a, b, c in zip(ref.actor_critic.parameters(), fus.actor_critic.parameters(), p0):
        da, db = (a.detach() - c), (b.detach() - c)
        assert da.abs().max() > 0
        # Adam steps are ~lr per entry: a flipped near-zero gradient moves an entry by up to 2 lr per step
        bad = ((da - db).abs() > 0.2 * lr).float().mean().item()
        assert bad < 0.02, bad
        assert (da - db).abs().max() <= 4 * 3 * lr


def test_loss_in_forward_launch_matches_the_separate_loss_kernel(monkeypatch):
    """pmlp_mlp_forward_ppo_loss (the loss in the update forward's launch, mini-batches of at
    least 18,432 rows) against the separate pmlp_ppo_loss_step launch (PMLP_FUSED_LOSS=0), one
    optimizer step from identical weights and rollout: both nets' output gradients bitwise (the
    same per-row arithmetic), the logged losses and every parameter to rounding (the partial
    sums run over 96-row instead of 64-row groups)."""
    torch.manual_seed(0)
    N, T, O, A = 1024, 24, 48, 12  # one mini-batch of 24,576 rows
    kw = dict(num_learning_epochs=1, num_mini_batches=1, learning_rate=1e-3, schedule="adaptive", device="cuda")
    ac0 = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
    algs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("PMLP_FUSED_LOSS", fused)
        alg = PPO(copy.deepcopy(ac0), **kw)
        alg.init_storage(N, T, [O], [None], [A])
        assert alg._fused is not None and alg._fused.fused_loss == (fused == "1")
        algs.append(alg)
    data = _fill_storage(algs[0], T, N, O, A, seed=3)
    for alg in algs:
        for k, v in data.items():
            getattr(alg.storage, k).copy_(v)
        alg.storage.step = T
    losses = []
    for alg in algs:
        torch.manual_seed(7)
        losses.append(alg.update())
    sep, fus = algs
    for n in range(2):
        assert torch.equal(fus._fused.dz_out[n], sep._fused.dz_out[n])
    np.testing.assert_allclose(losses[1], losses[0], rtol=1e-5, atol=1e-7)
    assert fus.learning_rate == pytest.approx(sep.learning_rate, rel=1e-6)
    for a, b in zip(sep.actor_critic.parameters(), fus.actor_critic.parameters()):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)


def test_adam_kernel_matches_torch_adam_with_clipping():
    """pmlp_opt_prepare + pmlp_adam == nn.utils.clip_grad_norm_ + torch.optim.Adam (fp32)
    over several steps with changing gradients, on flat buffers."""
    lib = mfma_mlp.load()
    torch.manual_seed(0)
    n = 100_003
    p_ref = torch.nn.Parameter(torch.randn(n, device="cuda"))
    lr = torch.tensor(3e-3, device="cuda")
    opt = torch.optim.Adam([p_ref], lr=3e-3)
    p = p_ref.detach().clone()
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    step = torch.zeros((), device="cuda")
    part = torch.empty(lib.pmlp_opt_parts(), device="cuda")
    for it in range(5):
        g = torch.randn(n, device="cuda") * (0.5 if it % 2 else 0.002)  # clipped and unclipped steps
        p_ref.grad = g.clone()
        torch.nn.utils.clip_grad_norm_([p_ref], 1.0)
        opt.step()
        s = mfma_mlp._stream()
        P = mfma_mlp._p
        mfma_mlp._ok(lib.pmlp_opt_prepare(P(g), n, 1.0, P(part), P(step), None, P(lr), None, 0.0, 0, s), "prep")
        mfma_mlp._ok(lib.pmlp_adam(P(p), P(g), P(m), P(v), n, 1.0, P(part), P(step), P(lr), 1.0, 0.9, 0.999, 1e-8, s),
                     "adam")
        torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)
        st = opt.state[p_ref]
        torch.testing.assert_close(m, st["exp_avg"], rtol=1e-5, atol=1e-8)
        torch.testing.assert_close(v, st["exp_avg_sq"], rtol=1e-5, atol=1e-10)
    assert float(step) == 5.0


@pytest.mark.parametrize("T,N", [(24, 4096), (7, 333)])
def test_gae_kernel_matches_storage_compute_returns(T, N):
    torch.manual_seed(0)
    sts = [RolloutStorage(N, T, [3], [None], [2], "cuda") for _ in range(2)]
    g = torch.Generator(device="cuda").manual_seed(3)
    rew = torch.randn(T, N, 1, device="cuda", generator=g)
    done = torch.rand(T, N, 1, device="cuda", generator=g) < 0.1
    val = torch.randn(T, N, 1, device="cuda", generator=g)
    last = torch.randn(N, 1, device="cuda", generator=g)
    for st in sts:
        st.rewards.copy_(rew)
        st.dones.copy_(done)
        st.values.copy_(val)
    sts[0].compute_returns(last, 0.99, 0.95)
    fused_step.gae(sts[1], last, 0.99, 0.95)
    torch.testing.assert_close(sts[1].returns, sts[0].returns, rtol=0, atol=1e-5)
    torch.testing.assert_close(sts[1].advantages, sts[0].advantages, rtol=0, atol=1e-4)


def test_fused_update_graph_is_bitwise_eager():
    """Replaying the captured fused update == running the same fused steps eagerly."""
    torch.manual_seed(0)
    N, T, O, A = 2048, 8, 48, 12
    ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
    algs = []
    for graph in (True, False):
        alg = PPO(copy.deepcopy(ac), num_learning_epochs=2, num_mini_batches=2, learning_rate=1e-3,
                  schedule="adaptive", device="cuda")
        alg.use_graph = graph
        alg.init_storage(N, T, [O], [None], [A])
        algs.append(alg)
    for u in range(4):
        data = _fill_storage(algs[1], T, N, O, A, seed=10 + u)
        for k, v in data.items():
            getattr(algs[0].storage, k).copy_(v)
        algs[0].storage.step = T
        torch.manual_seed(100 + u)
        lg = algs[0].update()
        torch.manual_seed(100 + u)
        le = algs[1].update()
        assert lg == le
        for a, b in zip(algs[0].actor_critic.parameters(), algs[1].actor_critic.parameters()):
            assert torch.equal(a, b)
    assert algs[0]._fgraph is not None and algs[1]._fgraph is None


def test_fused_checkpoint_roundtrip(tmp_path):
    """state_dicts keep the reference structure and a reload lands in the flat buffers."""
    torch.manual_seed(0)
    N, T, O, A = 512, 8, 48, 12
    alg = PPO(ActorCritic(O, O, A, [128, 64], [128, 64]).cuda(), num_learning_epochs=1, num_mini_batches=2,
              device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    _fill_storage(alg, T, N, O, A, seed=2)
    alg.update()
    path = tmp_path / "ck.pt"
    torch.save({"model_state_dict": alg.actor_critic.state_dict(),
                "optimizer_state_dict": alg.optimizer.state_dict()}, path)
    ck = torch.load(path, map_location="cuda", weights_only=True)
    assert set(ck["model_state_dict"]) == set(alg.actor_critic.state_dict())
    alg2 = PPO(ActorCritic(O, O, A, [128, 64], [128, 64]).cuda(), num_learning_epochs=1, num_mini_batches=2,
               device="cuda")
    alg2.init_storage(N, T, [O], [None], [A])
    alg2.actor_critic.load_state_dict(ck["model_state_dict"])
    alg2.optimizer.load_state_dict(ck["optimizer_state_dict"])
    alg2._fused.sync_optimizer_state(alg2.optimizer)
    for a, b in zip(alg.actor_critic.parameters(), alg2.actor_critic.parameters()):
        assert torch.equal(a, b)
    torch.testing.assert_close(alg2._fused.exp_avg, alg._fused.exp_avg)
    torch.testing.assert_close(alg2._fused.exp_avg_sq, alg._fused.exp_avg_sq)
    assert float(alg2._fused.step_t) == float(alg._fused.step_t) == 2.0


def test_fused_rollout_act_and_store_match_reference_semantics():
    """PPO.act / process_env_step through FusedRollout: actions ~ N(mu, std) (sample
    moments), log-prob, mean, sigma, value and observations in the storage row exactly
    as the reference computes them from the same policy outputs; the time-out bootstrap
    bitwise as the torch statement (deferred into the next act's launch, the last one
    flushed before the storage is read); fresh noise every step."""
    from torch.distributions import Normal
    torch.manual_seed(0)
    N, T, O, A = 4096, 4, 48, 12
    alg = PPO(ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda(), device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    assert alg._rollout is not None
    ac, st = alg.actor_critic, alg.storage
    g = torch.Generator(device="cuda").manual_seed(4)
    prev = None
    with torch.inference_mode():
        for t in range(T):
            obs = torch.randn(N, O, device="cuda", generator=g)
            actions = alg.act(obs, obs).clone()
            mu, value = alg._rollout.out  # the policy outputs of this act()
            torch.testing.assert_close(st.mu[t], mu, rtol=0, atol=0)
            torch.testing.assert_close(st.values[t], value, rtol=0, atol=0)
            with torch.no_grad():  # bf16 operands, fp32 accumulation vs the fp32 torch MLPs
                mu32, v32 = ac.actor.float()(obs), ac.critic.float()(obs)
            assert (mu - mu32).abs().max() <= 2e-2 * mu32.abs().max()
            assert (value - v32).abs().max() <= 2e-2 * v32.abs().max()
            torch.testing.assert_close(st.observations[t], obs, rtol=0, atol=0)
            sig = (mu * 0.0 + ac.std).detach()
            torch.testing.assert_close(st.sigma[t], sig, rtol=0, atol=0)
            assert torch.equal(st.actions[t], actions)
            z = (actions - mu) / sig
            assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1.0) < 0.01
            lp = Normal(mu, sig).log_prob(actions).sum(dim=-1)
            torch.testing.assert_close(st.actions_log_prob[t].squeeze(1), lp, rtol=1e-5, atol=1e-4)
            if prev is not None:
                assert not torch.equal(z, prev)
            prev = z
            rew = torch.randn(N, device="cuda", generator=g)
            done = torch.rand(N, device="cuda", generator=g) < 0.1
            tout = done & (torch.rand(N, device="cuda", generator=g) < 0.5)
            if t > 0:  # the previous step's store rode in this act's launch
                assert torch.equal(st.rewards[t - 1].squeeze(1), refs[-1][0])
                assert torch.equal(st.dones[t - 1].squeeze(1), refs[-1][1])
            alg.process_env_step(rew, done, {"time_outs": tout})
            ref = rew.clone()
            ref += alg.gamma * torch.squeeze(value.clone() * tout.unsqueeze(1), 1)
            refs = [(ref, done.clone())]
    alg.flush_rollout()
    assert torch.equal(st.rewards[T - 1].squeeze(1), refs[-1][0])
    assert torch.equal(st.dones[T - 1].squeeze(1), refs[-1][1])
    assert st.step == T
    with pytest.raises(AssertionError):
        alg.act(obs, obs)


def test_compute_returns_last_values_are_bitwise_evaluate():
    """compute_returns takes the last values from one launch of the critic's fused forward
    (FusedRollout.values) instead of ActorCritic.evaluate's layer GEMMs: the same bits, and
    the same GAE results as the evaluate path."""
    torch.manual_seed(0)
    N, T, O, A = 4096, 4, 48, 12
    alg = PPO(ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda(), device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    assert isinstance(alg._rollout, fused_step.FusedRollout)
    g = torch.Generator(device="cuda").manual_seed(9)
    cobs = torch.randn(N, O, device="cuda", generator=g)
    with torch.inference_mode():
        v = alg._rollout.values(cobs).clone()
        ref = alg.actor_critic.evaluate(cobs).detach()
    assert v.shape == ref.shape and torch.equal(v, ref)
    st = alg.storage
    for k in ("values", "rewards"):
        getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
    st.dones.copy_(torch.rand(st.dones.shape, device="cuda", generator=g) < 0.1)
    st.step = T
    with torch.inference_mode():
        alg.compute_returns(cobs)
    got = (st.returns.clone(), st.advantages.clone())
    ro, alg._rollout = alg._rollout, None  # the evaluate path
    with torch.inference_mode():
        alg.compute_returns(cobs)
    alg._rollout = ro
    assert torch.equal(got[0], st.returns) and torch.equal(got[1], st.advantages)


@pytest.mark.parametrize("K,ks", [(24576, 1152), (1000, 320)])
def test_partial_tn_gemm_matches_transposed_partial_and_fp32(K, ks):
    """Weight-gradient GEMM read from the row-major activations (PARTIAL_TN, LDS-transposed
    MFMA operands) == the k-contiguous PARTIAL on transposed copies, bitwise (same k order
    into the same MFMAs), and == fp32 dz^T y within fp32 summation order."""
    g = torch.Generator(device="cuda").manual_seed(3)
    for M, N in ((512, 56), (256, 520), (128, 264), (12, 136), (1, 136), (64, 64)):
        mp, np_ = (M + 7) // 8 * 8, (N + 7) // 8 * 8
        a = torch.randn(K, mp, device="cuda", generator=g).to(torch.bfloat16)
        b = torch.randn(K, np_, device="cuda", generator=g).to(torch.bfloat16)
        nsl = (K + ks - 1) // ks
        s_tn = torch.full((nsl, M, N), float("nan"), device="cuda")
        s_nt = torch.full((nsl, M, N), float("nan"), device="cuda")
        at, bt = a.t().contiguous(), b.t().contiguous()
        kp = (K + 7) // 8 * 8
        if kp != K:  # the NT path needs k padded to 8 (zeros)
            at = torch.nn.functional.pad(at, (0, kp - K))
            bt = torch.nn.functional.pad(bt, (0, kp - K))
        mfma_mlp._gemm(mfma_mlp.EPI_PARTIAL_TN, [dict(A=a, B=b, M=M, N=N, K=K, cf=s_tn)], ksplit=ks)
        mfma_mlp._gemm(mfma_mlp.EPI_PARTIAL, [dict(A=at, B=bt, M=M, N=N, K=kp, cf=s_nt)], ksplit=ks)
        torch.cuda.synchronize()
        assert torch.isfinite(s_tn).all(), (M, N)
        assert torch.equal(s_tn, s_nt), (M, N, float((s_tn - s_nt).abs().max()))
        ref = a[:, :M].float().t() @ b[:, :N].float()
        err = float((s_tn.sum(0) - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, (M, N, err)


@pytest.mark.parametrize("K,ks", [(24576, 1536), (1000, 320)])
def test_partial_tn_sum_col_is_the_ones_column_product(K, ks):
    """sum_col (the bias gradient from the A fragments times a ones operand) == the
    product with a column of ones appended to B, bitwise, and the weight columns are
    unchanged; column tiles no longer include the ones column."""
    g = torch.Generator(device="cuda").manual_seed(5)
    for M, n in ((512, 48), (256, 512), (128, 256), (12, 128), (1, 128), (64, 56)):
        mp = (M + 7) // 8 * 8
        a = torch.randn(K, mp, device="cuda", generator=g).to(torch.bfloat16)
        b = torch.zeros(K, n + 8, device="cuda", dtype=torch.bfloat16)
        b[:, :n] = torch.randn(K, n, device="cuda", generator=g).to(torch.bfloat16)
        b[:, n] = 1.0
        nsl = (K + ks - 1) // ks
        s_col = torch.full((nsl, M, n + 8), float("nan"), device="cuda")
        s_sum = torch.full((nsl, M, n + 8), float("nan"), device="cuda")
        mfma_mlp._gemm(mfma_mlp.EPI_PARTIAL_TN, [dict(A=a, B=b, M=M, N=n + 8, K=K, cf=s_col)], ksplit=ks)
        mfma_mlp._gemm(mfma_mlp.EPI_PARTIAL_TN, [dict(A=a, B=b, M=M, N=n, K=K, cf=s_sum, sum_col=n)], ksplit=ks)
        torch.cuda.synchronize()
        assert torch.equal(s_sum[..., :n + 1], s_col[..., :n + 1]), (M, n)
        assert torch.isnan(s_sum[..., n + 1:]).all()  # nothing past the bias column written
        ref = a[:, :M].float().sum(0)
        err = float((s_sum[..., n].sum(0) - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, (M, n, err)


@pytest.mark.parametrize("M,A,Ap", [(24576, 12, 16), (1000 + 37, 12, 16), (517, 8, 8), (2048, 10, 16)])
def test_loss_step_kernel_matches_fp32_autograd(M, A, Ap):
    """pmlp_ppo_loss_step (the quad-per-row kernel for A % 4 == 0, the one-lane-per-row
    kernel for A = 10) against rsl_rl v1.0.2's loss statement in fp32 autograd, rollout
    inputs gathered through a mini-batch index: the logged statistics, the std gradient
    (with the entropy term) and the bf16 output gradients of mu and the value."""
    g = torch.Generator(device="cuda").manual_seed(M + A)
    dev, R, clip, vcoef, ecoef = "cuda", M + 311, 0.2, 1.0, 0.01
    rn = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    mu = rn(M, A)
    std = 0.5 + torch.rand(A, device=dev, generator=g)
    value = rn(M, 1)
    act, old_mu = rn(R, A), rn(R, A)
    old_sigma = 0.5 + torch.rand(R, A, device=dev, generator=g)
    adv, ret = rn(R, 1), rn(R, 1)
    target = ret + 0.3 * rn(R, 1)
    rows = torch.randperm(R, device=dev, generator=g)[:M].contiguous()
    # old log-probs near the current ones: ratios spread across the clip range
    old_logp = rn(R, 1)
    old_logp[rows] = (torch.distributions.Normal(mu, std).log_prob(act[rows]).sum(-1, keepdim=True)
                      + 0.15 * rn(M, 1))

    # torch statement (rsl_rl v1.0.2 PPO.update, clipped value loss)
    tm, ts, tv = (t.clone().requires_grad_(True) for t in (mu, std, value))
    ga = lambda t: t[rows]  # noqa: E731
    dist = torch.distributions.Normal(tm, tm * 0 + ts)
    logp = dist.log_prob(ga(act)).sum(-1)
    ratio = torch.exp(logp - ga(old_logp).squeeze(-1))
    a_ = ga(adv).squeeze(-1)
    surr = torch.max(-a_ * ratio, -a_ * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    tgt, rt = ga(target), ga(ret)
    vc = tgt + (tv - tgt).clamp(-clip, clip)
    vl = torch.max((tv - rt).pow(2), (vc - rt).pow(2)).mean()
    ent = dist.entropy().sum(-1).mean()
    (surr + vcoef * vl - ecoef * ent).backward()
    with torch.no_grad():
        os_, om = ga(old_sigma), ga(old_mu)
        kl = torch.sum(torch.log(ts / os_ + 1e-5) + (os_ ** 2 + (om - tm) ** 2) / (2 * ts ** 2) - 0.5, -1).mean()

    L = mfma_mlp.load()
    P = mfma_mlp._p
    Vp = 8
    partial = torch.empty(L.pmlp_ppo_loss_step_parts(M, A), device=dev)
    stats, dstd = torch.empty(4, device=dev), torch.empty(A, device=dev)
    dmu = torch.full((M, Ap), float("nan"), dtype=torch.bfloat16, device=dev)
    dv = torch.full((M, Vp), float("nan"), dtype=torch.bfloat16, device=dev)
    mfma_mlp._ok(L.pmlp_ppo_loss_step(P(mu), P(std), P(value), P(act), P(old_logp), P(old_mu), P(old_sigma), P(adv),
                                      P(ret), P(target), P(rows), M, A, clip, 1, vcoef, ecoef, P(partial), P(stats),
                                      P(dstd), P(dmu), None, Ap, P(dv), None, Vp, mfma_mlp._stream()),
                 "pmlp_ppo_loss_step")
    torch.cuda.synchronize()
    want = torch.stack([surr.detach(), vl.detach(), kl, ent.detach()])
    torch.testing.assert_close(stats, want, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dstd, ts.grad, rtol=1e-4, atol=1e-7)
    # bf16 outputs: one rounding of the fp32 gradient; padding columns exactly zero
    torch.testing.assert_close(dmu[:, :A].float(), tm.grad.to(torch.bfloat16).float(), rtol=8e-3, atol=1e-9)
    assert torch.count_nonzero(dmu[:, A:].float()) == 0
    torch.testing.assert_close(dv[:, :1].float(), tv.grad.to(torch.bfloat16).float(), rtol=8e-3, atol=1e-9)
    assert torch.count_nonzero(dv[:, 1:].float()) == 0


def test_refused_update_capture_falls_back_to_the_eager_update(monkeypatch):
    """A capture that raises (as a collective library refusing capture would) leaves the
    update eager and training: the update runs, parameters move, no graph is kept; the same
    for the recurrent (autograd) update graph."""
    from contextlib import contextmanager
    from rsl_rl.modules import ActorCriticRecurrent

    @contextmanager
    def refused(*a, **k):
        raise RuntimeError("capture refused (test)")
        yield  # noqa

    torch.manual_seed(0)
    N, T, O, A = 512, 8, 48, 12
    alg = PPO(ActorCritic(O, O, A, [128, 64], [128, 64]).cuda(), num_learning_epochs=1, num_mini_batches=2,
              device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    _fill_storage(alg, T, N, O, A, seed=4)
    alg.update()  # eager first call
    monkeypatch.setattr(torch.cuda, "graph", refused)
    _fill_storage(alg, T, N, O, A, seed=5)
    p0 = [p.detach().clone() for p in alg.actor_critic.parameters()]
    with pytest.warns(UserWarning, match="capturing the update failed"):
        losses = alg.update()
    assert alg._fgraph is None and not alg.use_graph and np.isfinite(losses).all()
    assert any(not torch.equal(p, q) for p, q in zip(alg.actor_critic.parameters(), p0))
    # recurrent: the warm-up pass is undone, then the eager update runs once
    ac = ActorCriticRecurrent(O, O + 3, A, actor_hidden_dims=[32], critic_hidden_dims=[32], rnn_type="lstm",
                              rnn_hidden_size=64, rnn_num_layers=1).cuda()
    ralg = PPO(ac, num_learning_epochs=1, num_mini_batches=2, device="cuda")
    ralg.init_storage(N, T, [O], [O + 3], [A])
    assert ralg.use_graph
    for it in range(2):
        st = ralg.storage
        g = torch.Generator(device="cuda").manual_seed(it)
        for k in ("observations", "privileged_observations", "actions", "mu", "values", "rewards"):
            getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
        st.sigma.fill_(1.0)
        st.actions_log_prob.copy_(torch.distributions.Normal(st.mu, st.sigma).log_prob(st.actions).sum(-1, keepdim=True))
        st.hidden_state_slots(0, [(1, N, 64)] * 2, [(1, N, 64)] * 2)
        st.step = T
        ralg.compute_returns(torch.randn(N, O + 3, device="cuda", generator=g))
        p0 = [p.detach().clone() for p in ac.parameters()]
        if it == 1:
            with pytest.warns(UserWarning, match="capturing the update failed"):
                losses = ralg.update()
            assert ralg._graph is None and not ralg.use_graph
        else:
            losses = ralg.update()
        assert np.isfinite(losses).all()
        assert any(not torch.equal(p, q) for p, q in zip(ac.parameters(), p0))


def test_deep_mlp_keeps_the_autograd_update():
    """More Linear layers per net than the Adam mirror takes (PMLP_MAX_MIRROR jobs): the fused
    step is refused at construction and the autograd update trains instead."""
    torch.manual_seed(0)
    N, T, O, A = 256, 8, 48, 12
    hid = [64, 64, 64, 64]  # 5 Linear layers per net: 10 bf16 weight copies > 8
    alg = PPO(ActorCritic(O, O, A, hid, hid).cuda(), num_learning_epochs=1, num_mini_batches=2, device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    assert alg._fused is None
    _fill_storage(alg, T, N, O, A, seed=6)
    p0 = [p.detach().clone() for p in alg.actor_critic.parameters()]
    assert np.isfinite(alg.update()).all()
    assert all(not torch.equal(p, q) for p, q in zip(alg.actor_critic.parameters(), p0))


def test_load_between_learn_calls_reaches_the_captured_rollout(tmp_path):
    """OnPolicyRunner.load() after the rollout graph was captured: the next replayed rollout
    samples from the LOADED policy (the graph reads the bf16 weight copies, which the runner
    refreshes before the replay), not from the weights the copies held before the load."""
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry
    from legged_gym.utils import get_args
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    args = get_args(["--task", "go2", "--num_envs", "512", "--headless"])
    env, _ = task_registry.make_env(name="go2", args=args)
    _, train_cfg = task_registry.get_cfgs("go2")
    cfg = class_to_dict(train_cfg)
    torch.manual_seed(1)
    donor = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
    with torch.no_grad():
        for p in donor.alg.actor_critic.actor.parameters():
            p.mul_(-1.5)  # far from the runner's own policy
    path = str(tmp_path / "ck.pt")
    donor.save(path)
    want_actor = copy.deepcopy(donor.alg.actor_critic.actor).float()
    torch.manual_seed(2)
    runner = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
    runner.learn(2)
    assert runner._rollout_graph is not None
    runner.load(path)
    runner.learn(1)  # replays the captured rollout, then updates
    st = runner.alg.storage
    with torch.no_grad():
        mu = want_actor(st.observations[:4].reshape(-1, st.observations.shape[-1]))
    torch.testing.assert_close(st.mu[:4].reshape(mu.shape), mu, rtol=0.05, atol=0.05)  # bf16 GEMMs


@pytest.mark.parametrize("M,rows", [(24576, True), (4096, False), (1000, True), (37, False)])
def test_fused_mlp_forward_is_bitwise_the_per_layer_gemms(M, rows):
    """pmlp_mlp_forward (both nets' 4 layers in one launch, activations in LDS) == the
    per-layer pmlp_gemm forward (af gather/convert, FWD_HIDDEN x3, FWD_OUT) bitwise: the
    converted input rows, every hidden output and both outputs; ragged M included; the
    weights read row-major (W) and fragment-packed (Wf, the Adam mirror's second copy)."""
    torch.manual_seed(0)
    N, T, O, A = 1024, 24, 48, 12
    alg = PPO(ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda(), num_learning_epochs=1,
              num_mini_batches=1, device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    f = alg._fused
    assert f.fused_fwd and f.wf is not None
    f.ensure_weights()
    g = torch.Generator(device="cuda").manual_seed(M)
    x = 2.0 * torch.randn(T * N, O, device="cuda", generator=g)
    idx = torch.randperm(T * N, device="cuda", generator=g)[:M] if rows else None
    outs = {}
    for fused in ("frag", True, False):
        y = [[torch.full((M, lin.out_features), float("nan"), dtype=torch.bfloat16, device="cuda") for lin in ls[:-1]]
             for ls in f.lins]
        out = [torch.full((M, ls[-1].out_features), float("nan"), device="cuda") for ls in f.lins]
        xa = torch.full((M, f.k0p[0]), float("nan"), dtype=torch.bfloat16, device="cuda")
        if fused:
            mfma_mlp.mlp_forward([dict(x=x, kx=O, rows=idx, xa=xa if n == 0 else None, K0=f.k0p[n], W=f.wb[n],
                                       Wf=f.wf[n] if fused == "frag" else None,
                                       b=[lin.bias.detach() for lin in f.lins[n]],
                                       N=[lin.out_features for lin in f.lins[n]], y=y[n], out=out[n])
                                  for n in range(2)], M)
        else:
            for l in range(4):
                last = l == 3
                gj = []
                for n in range(2):
                    lin = f.lins[n][l]
                    a = dict(af=x, rows=idx, xa=xa if n == 0 else None) if l == 0 else dict(A=y[n][l - 1])
                    o = dict(cf=out[n]) if last else dict(cb=y[n][l])
                    gj.append(dict(B=f.wb[n][l], M=M, N=lin.out_features, K=f.k0p[n] if l == 0 else lin.in_features,
                                   bias=lin.bias.detach(), **a, **o))
                mfma_mlp._gemm(mfma_mlp.EPI_FWD_OUT if last else mfma_mlp.EPI_FWD_HIDDEN, gj)
        torch.cuda.synchronize()
        outs[fused] = (xa, y, out)
    for form in ("frag", True):
        (xa1, y1, o1), (xa0, y0, o0) = outs[form], outs[False]
        assert torch.equal(xa1, xa0)
        for n in range(2):
            for a, b in zip(y1[n], y0[n]):
                assert torch.equal(a, b)
            assert torch.equal(o1[n], o0[n])


def test_adam_mirror_writes_the_fragment_packed_weights():
    """After fused optimizer steps, the Adam mirror's fragment-packed copies (pmlp_mirror_job
    .frag) equal frag_pack of its row-major bf16 copies, which equal bf16 of the fp32 weights."""
    torch.manual_seed(0)
    N, T, O, A = 512, 24, 48, 12
    alg = PPO(ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda(), num_learning_epochs=1,
              num_mini_batches=2, device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    st = alg.storage
    g = torch.Generator(device="cuda").manual_seed(3)
    for k in ("observations", "actions", "values", "returns", "advantages", "mu"):
        getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
    st.sigma.fill_(1.0)
    st.actions_log_prob.copy_(-12.0 + torch.randn(st.actions_log_prob.shape, device="cuda", generator=g))
    st.step = T
    f = alg._fused
    assert f.wf is not None
    alg.use_graph = False
    alg.update()
    torch.cuda.synchronize()
    assert not f.weights_changed
    for n in range(2):
        for l, lin in enumerate(f.lins[n]):
            wb, wf = f.wb[n][l], f.wf[n][l]
            assert torch.equal(wb[:lin.out_features, :lin.in_features], lin.weight.detach().to(torch.bfloat16))
            assert torch.equal(wf, mfma_mlp.frag_pack(wb, wf.numel() // wb.shape[1]))


@pytest.mark.parametrize("n", [1, 7, 4096, 98304, 100003])
def test_minibatch_permutation_kernel_is_a_permutation(n):
    """pmlp_permutation (the fused update's mini-batch permutation in place of
    torch.randperm): every index of [0, n) exactly once, the same permutation for the same
    torch seed, a different one for the next draw, and no visible order left (the mean
    displacement of a uniform permutation is n/3)."""
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    torch.manual_seed(5)
    a = mfma_mlp.permutation_(out).clone()
    b = mfma_mlp.permutation_(out).clone()
    torch.manual_seed(5)
    c = mfma_mlp.permutation_(out).clone()
    assert torch.equal(torch.sort(a).values, torch.arange(n, device="cuda"))
    assert torch.equal(a, c)
    if n >= 4096:
        assert not torch.equal(a, b)
        disp = (a - torch.arange(n, device="cuda")).abs().double().mean().item()
        assert abs(disp - n / 3) < 0.02 * n


@pytest.mark.parametrize("T", [3, 4])
def test_fused_rollout_noise_is_fresh_across_iterations(T):
    """the draw-counter parity follows the acts, not the storage index, so
    with an odd num_steps_per_env the next iteration's first step does not reuse the last
    step's noise; every step of two iterations samples different noise."""
    torch.manual_seed(0)
    N, O, A = 1024, 48, 12
    alg = PPO(ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda(), device="cuda")
    alg.init_storage(N, T, [O], [None], [A])
    assert alg._rollout is not None
    st = alg.storage
    obs = torch.randn(N, O, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    zs = []
    for it in range(2):
        for t in range(T):
            with torch.inference_mode():
                a = alg.act(obs, obs).clone()
                zs.append(((a - alg._rollout.out[0]) / st.sigma[t]).clone())
                alg.process_env_step(torch.zeros(N, device="cuda"), torch.zeros(N, dtype=torch.bool, device="cuda"),
                                     {"time_outs": torch.zeros(N, dtype=torch.bool, device="cuda")})
        alg.flush_rollout()
        st.clear()
    for i in range(len(zs)):
        for j in range(i):
            assert (zs[i] == zs[j]).float().mean().item() < 0.01, (T, i, j)


@pytest.mark.parametrize("mlp", [[512, 256, 128], [256, 128, 64]])
def test_paired_backward_launch_is_bitwise_the_two_launches(monkeypatch, mlp):
    """pmlp_gemm_pair (a layer's weight gradient beside its input gradient in one grid)
    against the two pmlp_gemm launches (PMLP_GEMM_PAIR=0): two captured updates of the Go2
    shapes (24,576-row mini-batches, 4 optimizer steps each) from identical weights and rollout
    end with bitwise-identical parameters, gradients and Adam moments; and an MLP whose tiles
    do not pair falls back to the two launches."""
    torch.manual_seed(0)
    N, T, O, A = 4096, 24, 48, 12
    kw = dict(num_learning_epochs=2, num_mini_batches=2, learning_rate=1e-3, schedule="adaptive", device="cuda")
    ac0 = ActorCritic(O, O, A, mlp, mlp).cuda()
    algs = []
    for pair in ("0", "1"):
        monkeypatch.setenv("PMLP_GEMM_PAIR", pair)
        alg = PPO(copy.deepcopy(ac0), **kw)
        alg.init_storage(N, T, [O], [None], [A])
        assert alg._fused is not None and alg._fused.pair_backward == (pair == "1")
        algs.append(alg)
    data = _fill_storage(algs[0], T, N, O, A, seed=5)
    for it in range(2):
        for alg in algs:
            for k, v in data.items():
                getattr(alg.storage, k).copy_(v)
            alg.storage.step = T
            torch.manual_seed(11 + it)
            alg.update()
    two, one = algs
    for a, b in zip(two.actor_critic.parameters(), one.actor_critic.parameters()):
        assert torch.equal(a, b)
    assert torch.equal(two._fused.grad, one._fused.grad)
    assert torch.equal(two._fused.exp_avg, one._fused.exp_avg) and torch.equal(two._fused.exp_avg_sq, one._fused.exp_avg_sq)
