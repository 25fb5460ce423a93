"""rsl_rl v1.0.2 API semantics on CPU (the library is absent from the reference
tree, so PPO parity is unpinned; these pin the restated algorithm instead)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from fake_env import FakeEnv
from rsl_rl.algorithms import PPO
from rsl_rl.modules import ActorCritic, ActorCriticRecurrent
from rsl_rl.runners import OnPolicyRunner
from rsl_rl.storage import RolloutStorage
from rsl_rl.utils import split_and_pad_trajectories, unpad_trajectories


def test_actor_critic_shapes_and_distribution():
    ac = ActorCritic(48, 48, 12, [512, 256, 128], [512, 256, 128], init_noise_std=1.0)
    obs = torch.randn(32, 48)
    a = ac.act(obs)
    assert a.shape == (32, 12)
    lp = ac.get_actions_log_prob(a)
    ref = torch.distributions.Normal(ac.actor(obs), ac.std).log_prob(a).sum(-1)
    torch.testing.assert_close(lp, ref)
    assert ac.evaluate(obs).shape == (32, 1)
    assert torch.allclose(ac.action_std, torch.ones(32, 12))
    n_params = sum(p.numel() for p in ac.parameters())
    assert n_params == 380313  # Go2 MLP bucket = 1.52 MB fp32


def test_gae_matches_naive_recursion():
    T, N, g, lam = 6, 5, 0.99, 0.95
    st = RolloutStorage(N, T, [3], [None], [2])
    rng = np.random.default_rng(0)
    rew = rng.normal(size=(T, N, 1)).astype(np.float32)
    val = rng.normal(size=(T, N, 1)).astype(np.float32)
    done = (rng.uniform(size=(T, N, 1)) < 0.2)
    st.rewards[:] = torch.from_numpy(rew)
    st.values[:] = torch.from_numpy(val)
    st.dones[:] = torch.from_numpy(done.astype(np.uint8))
    last = rng.normal(size=(N, 1)).astype(np.float32)
    st.compute_returns(torch.from_numpy(last), g, lam)
    ret = np.zeros_like(rew)
    adv = np.zeros((N, 1), np.float32)
    for t in reversed(range(T)):
        nv = last if t == T - 1 else val[t + 1]
        nt = 1.0 - done[t].astype(np.float32)
        delta = rew[t] + nt * g * nv - val[t]
        adv = delta + nt * g * lam * adv
        ret[t] = adv + val[t]
    np.testing.assert_allclose(st.returns.numpy(), ret, rtol=1e-5, atol=1e-5)
    a = ret - val
    np.testing.assert_allclose(st.advantages.numpy(), (a - a.mean()) / (a.std(ddof=1) + 1e-8), rtol=1e-4, atol=1e-4)


def test_split_and_pad_roundtrip():
    T, N = 5, 3
    x = torch.arange(T * N * 2, dtype=torch.float).view(T, N, 2)
    dones = torch.zeros(T, N, 1, dtype=torch.uint8)
    dones[1, 0] = 1
    dones[3, 2] = 1
    padded, masks = split_and_pad_trajectories(x, dones)
    assert padded.shape[0] == T and masks.shape == (T, padded.shape[1])
    assert padded.shape[1] == 5  # env0: 2 trajs, env1: 1, env2: 2
    back = unpad_trajectories(padded, masks)
    torch.testing.assert_close(back, x)


def test_ppo_update_changes_params_and_adapts_lr():
    torch.manual_seed(0)
    env = FakeEnv(num_envs=32)
    ac = ActorCritic(env.num_obs, env.num_obs, env.num_actions, [32], [32])
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=2, learning_rate=1e-3, schedule="adaptive", desired_kl=0.01)
    ppo.init_storage(env.num_envs, 8, [env.num_obs], [None], [env.num_actions])
    obs, _ = env.reset()
    before = [p.detach().clone() for p in ac.parameters()]
    for _ in range(8):
        a = ppo.act(obs, obs)
        obs, _, r, d, info = env.step(a)
        ppo.process_env_step(r, d, info)
    ppo.compute_returns(obs)
    vl, sl = ppo.update()
    assert np.isfinite(vl) and np.isfinite(sl)
    assert any(not torch.equal(b, p) for b, p in zip(before, ac.parameters()))
    assert ppo.learning_rate != 1e-3  # KL-adaptive schedule moved it
    assert 1e-5 <= ppo.learning_rate <= 1e-2


def test_time_out_bootstrap_adds_gamma_value():
    env = FakeEnv(num_envs=4)
    ac = ActorCritic(env.num_obs, env.num_obs, env.num_actions, [8], [8])
    ppo = PPO(ac, gamma=0.9)
    ppo.init_storage(4, 2, [env.num_obs], [None], [env.num_actions])
    obs, _ = env.reset()
    ppo.act(obs, obs)
    v = ppo.transition.values.clone()
    r = torch.ones(4)
    to = torch.tensor([True, False, True, False])
    ppo.process_env_step(r, to, {"time_outs": to})
    torch.testing.assert_close(ppo.storage.rewards[0, :, 0], r + 0.9 * v[:, 0] * to)


def test_runner_learn_save_load(tmp_path):
    env = FakeEnv(num_envs=16, num_privileged_obs=9)
    cfg = {"runner": {"policy_class_name": "ActorCritic", "algorithm_class_name": "PPO", "num_steps_per_env": 8,
                      "save_interval": 1},
           "algorithm": {"num_learning_epochs": 1, "num_mini_batches": 2, "learning_rate": 1e-3},
           "policy": {"actor_hidden_dims": [16], "critic_hidden_dims": [16], "activation": "elu", "init_noise_std": 1.0}}
    runner = OnPolicyRunner(env, cfg, log_dir=str(tmp_path), device="cpu")
    runner.learn(2, init_at_random_ep_len=True)
    assert (tmp_path / "model_0.pt").exists() and (tmp_path / "model_2.pt").exists()
    ck = torch.load(tmp_path / "model_2.pt", weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "iter", "infos"} and ck["iter"] == 2
    r2 = OnPolicyRunner(env, cfg, log_dir=None, device="cpu")
    r2.load(str(tmp_path / "model_2.pt"))
    assert r2.current_learning_iteration == 2
    pol = r2.get_inference_policy()
    assert pol(env.get_observations()).shape == (16, env.num_actions)


def test_recurrent_runner_learns(tmp_path):
    env = FakeEnv(num_envs=8, num_privileged_obs=9, ep_len=5)
    cfg = {"runner": {"policy_class_name": "ActorCriticRecurrent", "algorithm_class_name": "PPO",
                      "num_steps_per_env": 12, "save_interval": 50},
           "algorithm": {"num_learning_epochs": 2, "num_mini_batches": 2},
           "policy": {"actor_hidden_dims": [16], "critic_hidden_dims": [16], "activation": "elu",
                      "rnn_type": "lstm", "rnn_hidden_size": 8, "rnn_num_layers": 1, "init_noise_std": 0.8}}
    runner = OnPolicyRunner(env, cfg, log_dir=None, device="cpu")
    runner.learn(2)
    assert runner.alg.actor_critic.is_recurrent


@pytest.mark.parametrize("robot", ["g1", "h1", "h1_2"])
def test_lstm_export_matches_pretrained_policy(robot, tmp_path):
    """Golden: deploy/pre_train/<robot>/motion.pt (the reference's own exported
    PolicyExporterLSTM).  Our ActorCriticRecurrent + PolicyExporterLSTM with the
    same weights must reproduce its outputs and its reset_memory semantics."""
    import legged_gym.envs  # noqa: F401  (train.py's import order: envs before utils)
    from legged_gym.utils.helpers import export_policy_as_jit
    g = np.load(os.path.join(GOLDEN, f"lstm_policy_{robot}.npz"))
    n_in = g["w.memory.weight_ih_l0"].shape[1]
    n_act = g["w.actor.2.weight"].shape[0]
    ac = ActorCriticRecurrent(n_in, n_in + 3, n_act, actor_hidden_dims=[32], critic_hidden_dims=[32],
                              rnn_type="lstm", rnn_hidden_size=64, rnn_num_layers=1, init_noise_std=0.8)
    sd = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w.")}
    ac.actor.load_state_dict({k[len("actor."):]: v for k, v in sd.items() if k.startswith("actor.")})
    ac.memory_a.rnn.load_state_dict({k[len("memory."):]: v for k, v in sd.items() if k.startswith("memory.")})
    export_policy_as_jit(ac, str(tmp_path))
    m = torch.jit.load(str(tmp_path / "policy_lstm_1.pt"))
    m.reset_memory()
    ys = np.stack([m(torch.from_numpy(x[None])).detach().numpy()[0] for x in g["inputs"]])
    np.testing.assert_allclose(ys, g["outputs"], rtol=1e-5, atol=1e-5)
    m.reset_memory()
    ys2 = np.stack([m(torch.from_numpy(x[None])).detach().numpy()[0] for x in g["inputs"][:5]])
    np.testing.assert_allclose(ys2, g["outputs_after_reset"], rtol=1e-5, atol=1e-5)
    # the training-time module computes the same recurrent forward
    ac.eval()
    ac.memory_a.hidden_states = None
    ys3 = np.stack([ac.act_inference(torch.from_numpy(x[None])).detach().numpy()[0] for x in g["inputs"]])
    np.testing.assert_allclose(ys3, g["outputs"], rtol=1e-5, atol=1e-5)


def test_splitk_linear_matches_linear_grads():
    """SplitKLinear (chunked weight gradient) == nn.Linear on CPU tensors via the same Function."""
    import torch
    from rsl_rl.modules import splitk_linear as skl
    torch.manual_seed(0)
    x = torch.randn(8192, 48, dtype=torch.float64, requires_grad=True)
    lin = torch.nn.Linear(48, 32).double()
    y = skl._SplitKLinearFn.apply(x, lin.weight, lin.bias)
    g = torch.randn_like(y)
    dx, dw, db = torch.autograd.grad(y, (x, lin.weight, lin.bias), g)
    y2 = torch.nn.functional.linear(x, lin.weight, lin.bias)
    dx2, dw2, db2 = torch.autograd.grad(y2, (x, lin.weight, lin.bias), g)
    assert torch.allclose(y, y2) and torch.allclose(dx, dx2) and torch.allclose(db, db2)
    assert torch.allclose(dw, dw2, rtol=1e-10, atol=1e-10)
    # state_dict keys identical to nn.Linear (checkpoints interchange)
    assert set(skl.SplitKLinear(48, 32).state_dict()) == set(lin.state_dict())


def test_dense_recurrent_update_equals_padded_trajectories():
    """The dense recurrent update (recurrent_dense_mini_batch_generator: every env's T steps with
    the LSTM state zeroed after dones) computes exactly rsl_rl v1.0.2's padded-trajectory update
    (reccurent_mini_batch_generator + split_and_pad_trajectories): same losses, same gradients."""
    torch.manual_seed(0)
    env = FakeEnv(num_envs=8, num_privileged_obs=9, ep_len=5)
    ac = ActorCriticRecurrent(6, 9, 3, actor_hidden_dims=[16], critic_hidden_dims=[16], rnn_type="lstm",
                              rnn_hidden_size=8, rnn_num_layers=1, init_noise_std=0.8)
    ppo = PPO(ac, num_learning_epochs=1, num_mini_batches=2, device="cpu")
    ppo.init_storage(8, 12, [6], [9], [3])
    obs, priv = env.reset()
    with torch.inference_mode():
        for it in range(2):  # two rollouts: the second starts from a carried (nonzero) state
            ppo.storage.clear()
            for _ in range(12):
                a = ppo.act(obs, priv)
                obs, priv, r, d, info = env.step(a)
                ppo.process_env_step(r, d, info)
            ppo.compute_returns(priv)
    st = ppo.storage
    assert st.dones.any() and st.saved_hidden_states_a[0][0].abs().sum() > 0
    params = list(ac.parameters())
    for (padded, dense) in zip(st.reccurent_mini_batch_generator(2, 1), st.recurrent_dense_mini_batch_generator(2, 1)):
        out = []
        for flag, batch in ((False, padded), (True, dense)):
            ppo._dense_recurrent = flag
            loss, surr, vl = ppo._reference_loss(*batch)
            out.append((loss.detach(), surr.detach(), vl.detach(), torch.autograd.grad(loss, params)))
        (l1, s1, v1, g1), (l2, s2, v2, g2) = out
        torch.testing.assert_close(l2, l1, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(s2, s1, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(v2, v1, rtol=1e-5, atol=1e-6)
        for a, b in zip(g2, g1):
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
    ppo._dense_recurrent = True


def test_recurrent_rollout_saves_pre_step_hidden_states():
    """The hidden state stored for step t is the state BEFORE step t (reset after dones)."""
    torch.manual_seed(1)
    env = FakeEnv(num_envs=4, ep_len=3)
    ac = ActorCriticRecurrent(6, 6, 3, actor_hidden_dims=[8], critic_hidden_dims=[8], rnn_type="lstm",
                              rnn_hidden_size=8, rnn_num_layers=1)
    ppo = PPO(ac, device="cpu")
    ppo.init_storage(4, 6, [6], [None], [3])
    obs, _ = env.reset()
    states = []
    with torch.inference_mode():
        for _ in range(6):
            hs = ac.get_hidden_states()
            states.append(None if hs[0] is None else hs[0][0].clone())
            a = ppo.act(obs, obs)
            obs, _, r, d, info = env.step(a)
            ppo.process_env_step(r, d, info)
    saved = ppo.storage.saved_hidden_states_a[0]  # [T, layers, N, H]
    for t in range(1, 6):
        torch.testing.assert_close(saved[t, 0], states[t][0])
    d = ppo.storage.dones[:, :, 0].bool()
    for t in range(1, 6):  # after a done the stored state is zero
        assert saved[t, 0][d[t - 1]].abs().sum() == 0


def test_gru_policy_trains_on_the_padded_generator():
    """ActorCriticRecurrent(rnn_type='gru'): the dense (LSTM-only) update form is not taken;
    the update runs rsl_rl's padded-trajectory generator and trains."""
    env = FakeEnv(num_envs=8, num_privileged_obs=9, ep_len=5)
    ac = ActorCriticRecurrent(6, 9, 3, actor_hidden_dims=[16], critic_hidden_dims=[16], rnn_type="gru",
                              rnn_hidden_size=8, rnn_num_layers=1)
    ppo = PPO(ac, num_learning_epochs=2, num_mini_batches=2, device="cpu")
    assert not ppo._dense_recurrent
    ppo.init_storage(8, 6, [6], [9], [3])
    obs, priv = env.reset()
    with torch.inference_mode():
        for _ in range(6):
            a = ppo.act(obs, priv)
            obs, priv, r, d, info = env.step(a)
            ppo.process_env_step(r, d, info)
        ppo.compute_returns(priv)
    p0 = [p.detach().clone() for p in ac.parameters()]
    losses = ppo.update()
    assert np.isfinite(losses).all()
    assert any(not torch.equal(p, q) for p, q in zip(ac.parameters(), p0))


def test_fused_step_refuses_nets_deeper_than_the_adam_mirror():
    """FusedPPOStep raises ValueError (which init_storage catches) for more Linear layers per
    net than PMLP_MAX_MIRROR / 2, before it allocates anything."""
    from rsl_rl.algorithms import fused_step
    from rsl_rl.modules import mfma_mlp
    hid = [16] * mfma_mlp.PMLP_MAX_MIRROR  # PMLP_MAX_MIRROR + 1 Linear layers per net
    ppo = PPO(ActorCritic(6, 6, 3, hid, hid), device="cpu")
    with pytest.raises(ValueError, match="Linear layers"):
        fused_step.FusedPPOStep(ppo, 64)


@pytest.mark.parametrize("hid,ok", [([32], True), ([16], True), ([12], False), ([20], False), ([28], False), ([40], False)])
def test_fused_recurrent_covers_only_head_widths_the_kernels_take(hid, ok):
    """pmlp_heads_forward / _backward take head hidden widths N0 <= 32 and a multiple of 8
    (lstm_seq.hip heads_check): any other width must keep the autograd update (supported()
    False) rather than build the fused step and fail at its first launch."""
    from rsl_rl.algorithms import fused_recurrent
    ac = ActorCriticRecurrent(47, 50, 12, actor_hidden_dims=hid, critic_hidden_dims=hid, rnn_type="lstm",
                              rnn_hidden_size=64, rnn_num_layers=1)
    assert fused_recurrent.supported(ac, 256, 4) is ok
