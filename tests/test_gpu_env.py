"""The env through its Python API (LeggedRobot on the C ABI): reset/push/time-out
semantics against the oracle, the VecEnv drop-in contract, the gymapi-style substep,
long rollouts, and the PPO paths on top of it.  The step-level bitwise parity of
the HIP kernel with the oracle (every robot, size and ground) is tests/test_gpu_parity.py.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
import bridge  # noqa: E402

TASKS = ["go2", "h1", "g1", "h1_2"]


def make(task, n, **edits):
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env_cfg, _ = task_registry.get_cfgs(task)
    import copy
    cfg = copy.deepcopy(env_cfg)
    for k, v in edits.items():
        sec, attr = k.split("__")
        setattr(getattr(cfg, sec), attr, v)
    env, _ = task_registry.make_env(name=task, args=args, env_cfg=cfg)
    return env


def compare(env, ref, keys, atol):
    n = env.num_envs
    got = {"root": env.root_states, "dofs": env.dof_state, "cforce": env._contact_forces, "obs": env.obs_buf,
           "priv_obs": env.privileged_obs_buf, "rew": env.rew_buf, "reset": env.reset_buf,
           "time_out": env.time_out_buf, "commands": env.commands, "episode_length": env._episode_length,
           "feet_air_time": env.feet_air_time, "last_contacts": env.last_contacts, "torques": env.torques,
           "episode_sums": env._episode_sums.T, "rbs": env.rigid_body_states}
    for k in keys:
        g = got[k].detach().cpu().numpy()
        r = ref[k]
        if k == "episode_sums":
            r = r.T
        if g.dtype == np.bool_:
            g = g.astype(np.uint8)
        bad = ~np.isclose(g.astype(np.float64), r.astype(np.float64), rtol=atol, atol=atol)
        nbad = int(bad.reshape(n, -1).any(axis=1).sum())
        assert np.isfinite(g).all(), k
        assert nbad == 0, f"{k}: {nbad}/{n} envs outside {atol} (max |d| {np.abs(g - r).max():.3e})"


@pytest.mark.parametrize("task", ["go2", "h1"])
def test_timeouts_reset_push_match_oracle_exactly(task):
    """Every env times out at once: the reset/push/resample draws (Philox) and the
    post-reset state must equal the oracle's; semantics of legged_robot.py:723-768."""
    env = make(task, 256)
    env.reset()
    env.step(torch.zeros(env.num_envs, env.num_actions, device="cuda"))
    env.episode_length_buf = torch.full_like(env.episode_length_buf, int(env.max_episode_length))
    snap = bridge.snapshot(env)
    a = torch.zeros(env.num_envs, env.num_actions, device="cuda")
    ref = bridge.step(env, snap, a.cpu().numpy(), env.common_step_counter)
    env.step(a)
    torch.cuda.synchronize()
    assert env.reset_buf.all() and env.time_out_buf.all()
    assert (env.episode_length_buf == 0).all()
    compare(env, ref, ["reset", "time_out", "episode_length", "commands", "root", "dofs", "episode_sums", "obs"],
            0.0)  # bit-exact (tests/test_gpu_parity.py)
    q = env.dof_pos / env.default_dof_pos
    m = env.default_dof_pos.abs().expand_as(q) > 1e-6
    assert ((q[m] >= 0.5 - 1e-6) & (q[m] <= 1.5 + 1e-6)).all()
    assert (env.dof_vel == 0).all()
    init = env.base_init_state
    torch.testing.assert_close(env.root_states[:, :3], init[:3] + env.env_origins)
    assert (env.root_states[:, 9:13].abs() <= 0.5).all()          # reset vel U[-0.5,0.5] (z, ang)
    v = env.cfg.domain_rand.max_push_vel_xy
    assert (env.root_states[:, 7:9].abs() <= v).all()              # pushed at ep_len 0
    ep = env.extras["episode"]
    assert set(ep) == {"rew_" + k for k in env._sum_names}
    assert env.extras["time_outs"].all()
    # extras["episode"] = sums over the reset envs / count / episode_length_s (:742-768)
    nsum = len(env._sum_names)
    acc = ref["episode_acc"]
    means = acc[:nsum] / max(float(acc[nsum]), 1.0) / env.max_episode_length_s
    got = torch.stack([ep["rew_" + k] for k in env._sum_names]).cpu().numpy()
    # float atomics over the reset envs: the sum order is not fixed
    np.testing.assert_allclose(got, means, rtol=1e-5, atol=1e-8)
    assert float(env._episode_acc.abs().sum()) == 0.0  # zeroed for the next step


def test_drop_in_semantics():
    env = make("go2", 64)
    obs, priv = env.reset()
    assert priv is None and obs.shape == (64, 48)
    assert env.num_obs == 48 and env.num_privileged_obs is None and env.num_actions == 12
    assert env.max_episode_length == 1000
    # rsl_rl rebinds episode_length_buf: values reach the kernel's buffer
    env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
    lens = env.episode_length_buf.clone()
    o1, _, r1, d1, x1 = env.step(torch.zeros(64, 12, device="cuda"))
    assert torch.equal(env.episode_length_buf[~d1], lens[~d1] + 1)
    kept = o1.clone()
    o2, _, r2, d2, x2 = env.step(torch.zeros(64, 12, device="cuda"))
    assert o2.data_ptr() != o1.data_ptr() and torch.equal(o1, kept)  # previous obs not overwritten
    assert d2.dtype == torch.bool and r2.dtype == torch.float32
    assert "time_outs" in x2 and "episode" in x2
    # stale extras when no env resets (legged_robot.py:742-743): a settled env (zero actions,
    # episode lengths held at 0, so no time-out and no fall) takes a step without a reset
    zero = torch.zeros(64, 12, device="cuda")
    for _ in range(10):
        env.episode_length_buf = torch.zeros_like(env.episode_length_buf)
        env.step(zero)
    env.episode_length_buf = torch.zeros_like(env.episode_length_buf)
    env.extras["time_outs"][:] = True
    prev = env.extras["time_outs"].clone()
    _, _, _, d3, x3 = env.step(zero)
    assert not d3.any()
    assert torch.equal(x3["time_outs"], prev)  # carried, not recomputed (all False otherwise)


def test_gymapi_style_substep_matches_oracle():
    """lgs_simulate (one substep with caller torques) == orc_simulate."""
    import ctypes as C
    from leggedsim import cabi
    env = make("go2", 128)
    env.reset()
    for _ in range(10):
        env.step(0.3 * torch.randn(128, 12, device="cuda"))
    tau = (5.0 * torch.randn(128, 12, device="cuda")).contiguous()
    snap = bridge.snapshot(env)
    env.sim.simulate(tau)
    torch.cuda.synchronize()
    lib = bridge.ensure_built()
    bridge.set_env(lib, env)
    mh = cabi.ModelHandle(env.model)
    root, dofs = snap["root"].copy(), snap["dofs"].copy()
    cf, rbs = snap["cforce"].copy(), snap["rbs"].copy()
    t = tau.cpu().numpy()
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_simulate(C.byref(mh.desc), C.byref(env._lgs_params), 128, p(root), p(dofs), p(t), p(cf), p(rbs),
                     p(snap["added_mass"]), p(snap["friction"]))
    np.testing.assert_array_equal(env.root_states.cpu().numpy(), root)  # bit-exact
    np.testing.assert_array_equal(env.dof_state.cpu().numpy(), dofs)


@pytest.mark.parametrize("task", TASKS)
def test_long_rollout_stays_finite(task):
    env = make(task, 256)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(300):
        env.step(torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g))
    torch.cuda.synchronize()
    for t in (env.root_states, env.dof_state, env.obs_buf, env.rew_buf):
        assert torch.isfinite(t).all()


def test_ppo_training_smoke():
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    env = make("go2", 512)
    _, train_cfg = task_registry.get_cfgs("go2")
    runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device="cuda:0")
    runner.learn(2, init_at_random_ep_len=True)
    for p in runner.alg.actor_critic.parameters():
        assert torch.isfinite(p).all()


def test_runner_without_device_syncs_trains_the_same_parameters():
    """OnPolicyRunner.learn without the device sync after the collection and without the loss
    read-back (no log directory: the host runs ahead of the device) trains bitwise the same
    parameters as with the syncs (sync_phase_times = True)."""
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    params = []
    for exact in (True, False):
        env = make("go2", 512)
        _, train_cfg = task_registry.get_cfgs("go2")
        runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device="cuda:0")
        runner.sync_phase_times = exact
        torch.manual_seed(123)
        runner.learn(3, init_at_random_ep_len=True)
        torch.cuda.synchronize()
        params.append([p.detach().clone() for p in runner.alg.actor_critic.parameters()])
    for a, b in zip(*params):
        assert torch.equal(a, b)


def test_recurrent_humanoid_training_smoke():
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    env = make("h1", 256)
    _, train_cfg = task_registry.get_cfgs("h1")
    runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device="cuda:0")
    runner.learn(1, init_at_random_ep_len=True)
    for p in runner.alg.actor_critic.parameters():
        assert torch.isfinite(p).all()


def test_ppo_update_graph_matches_eager():
    """The whole-update HIP graph performs the same optimizer steps as the eager loop.
    Fixed LR schedule: the adaptive schedule's x1.5 thresholds would amplify
    last-bit GEMM differences into different learning rates."""
    import copy
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    env = make("go2", 256)
    _, train_cfg = task_registry.get_cfgs("go2")
    cfg = class_to_dict(train_cfg)
    cfg["algorithm"]["schedule"] = "fixed"
    cfg["algorithm"]["learning_rate"] = 3e-4
    cfg["policy"]["mixed_precision"] = False  # fp32: both paths then run bit-comparable GEMMs
    # one optimizer step: its loss is computed before any parameter moves, so it
    # must agree to fp32 rounding; the step itself may differ by ~2 lr on
    # parameters whose gradient is ~0 (Adam normalises the sign of the noise)
    cfg["algorithm"]["num_learning_epochs"] = 1
    cfg["algorithm"]["num_mini_batches"] = 1
    runner = OnPolicyRunner(env, cfg, log_dir=None, device="cuda:0")
    runner.learn(2)  # eager warm-up update, then the captured graph
    alg = runner.alg
    assert alg.use_graph and alg._graph is not None
    with torch.inference_mode():
        obs = env.get_observations()
        for _ in range(alg.storage.num_transitions_per_env):
            a = alg.act(obs, obs)
            obs, _, r, d, info = env.step(a)
            alg.process_env_step(r, d, info)
        alg.compute_returns(obs)
    saved = {k: v.clone() for k, v in alg.storage.__dict__.items() if torch.is_tensor(v) and not k.startswith("_")}
    params = list(alg.actor_critic.parameters())
    p0 = [p.detach().clone() for p in params]
    st0 = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in alg.optimizer.state[p].items()} for p in params}
    torch.manual_seed(5)
    rng, rng_cpu = torch.cuda.get_rng_state(), torch.get_rng_state()
    g_losses = alg.update()  # graphed
    p_graph = [p.detach().clone() for p in params]
    with torch.no_grad():  # rewind IN PLACE (the graph holds these buffers)
        for p, v in zip(params, p0):
            p.copy_(v)
        for p in params:
            for k, v in alg.optimizer.state[p].items():
                if torch.is_tensor(v):
                    v.copy_(st0[id(p)][k])
        for k, v in saved.items():
            getattr(alg.storage, k).copy_(v)
    alg.storage.step = alg.storage.num_transitions_per_env
    torch.cuda.set_rng_state(rng)
    torch.set_rng_state(rng_cpu)
    alg.use_graph = False
    e_losses = alg.update()
    alg.use_graph = True
    np.testing.assert_allclose(g_losses, e_losses, rtol=1e-4, atol=1e-7)
    for a, b, c in zip(params, p_graph, p0):
        assert (a.detach() - b).abs().max() <= 2.5 * 3e-4
        assert (b - c).abs().max() > 0  # the graph really stepped


def test_ppo_graph_tracks_eager_over_many_updates():
    """The captured update (fp32) replayed on fresh rollouts each time stays finite
    and on the eager trajectory.  Guards two failure modes seen on this ROCm: a
    stale autograd graph pinning AccumulateGrad to another stream (replays race),
    and bf16 library GEMMs drifting inside the graph (mixed precision => eager)."""
    import copy
    from rsl_rl.algorithms import PPO
    from rsl_rl.modules import ActorCritic
    torch.manual_seed(0)
    N, T, O, A = 2048, 8, 48, 12  # 8192-row mini-batches: the split-K weight-gradient path
    ac = ActorCritic(O, O, A, [128, 64], [128, 64]).cuda()
    algs = []
    for graph in (True, False):
        alg = PPO(copy.deepcopy(ac), num_learning_epochs=2, num_mini_batches=2, learning_rate=1e-3,
                  schedule="fixed", device="cuda")
        alg.use_graph = graph
        alg.init_storage(N, T, [O], [None], [A])
        alg._rollout = None  # the reference act()/process_env_step: the test sets the actions itself
        algs.append(alg)
    g = torch.Generator(device="cuda").manual_seed(1)
    losses = {True: [], False: []}
    for u in range(12):
        obs = [torch.randn(N, O, device="cuda", generator=g) for _ in range(T + 1)]
        act = [torch.randn(N, A, device="cuda", generator=g) for _ in range(T)]
        rew = [0.1 * torch.randn(N, device="cuda", generator=g) for _ in range(T)]
        for alg in algs:
            with torch.inference_mode():
                for t in range(T):
                    alg.act(obs[t], obs[t])
                    alg.transition.actions = act[t]  # identical actions for both twins
                    alg.transition.actions_log_prob = alg.actor_critic.get_actions_log_prob(act[t]).detach()
                    alg.process_env_step(rew[t], torch.zeros(N, device="cuda", dtype=torch.bool), {})
                alg.compute_returns(obs[T])
            losses[alg.use_graph].append(alg.update())
        pg, pe = (list(a.actor_critic.parameters()) for a in algs)
        assert all(torch.isfinite(p).all() for p in pg), f"graphed update went non-finite at update {u}"
        # Adam turns rounding-level gradient differences into <= ~lr moves per step
        d = max(float((x - y).abs().max()) for x, y in zip(pg, pe))
        assert d < 2 * 1e-3 * 4 * (u + 1), f"update {u}: graphed params drifted {d:.3e} from eager"
    assert algs[0]._graph is not None or algs[0]._fgraph is not None
    # the failure mode seen before the fixes: the graph optimised systematically worse
    vg, sg = np.array(losses[True]).T
    ve, se = np.array(losses[False]).T
    assert abs(vg.mean() - ve.mean()) <= 0.05 * abs(ve.mean()), (vg, ve)
    assert abs(sg.mean() - se.mean()) <= 0.2 * abs(se.mean()) + 1e-4, (sg, se)


@pytest.mark.parametrize("rows", [4096, 24576, 200])
def test_mfma_mlp_matches_fp32_torch(rows):
    """bf16-MFMA MLP (csrc/ppo_mlp.hip) vs the same nn.Sequential in fp32 torch:
    outputs and every parameter gradient within bf16 rounding (relative 2e-2)."""
    from rsl_rl.modules import mfma_mlp
    from rsl_rl.modules.actor_critic import mlp, get_activation
    torch.manual_seed(0)
    for out_dim, in_dim in ((12, 48), (1, 47)):
        net = mlp(in_dim, [512, 256, 128], out_dim, get_activation("elu")).cuda()
        x = torch.randn(rows, in_dim, device="cuda")
        y_ref = net(x)
        g = torch.randn_like(y_ref)
        grads_ref = torch.autograd.grad(y_ref, list(net.parameters()), g)
        if not mfma_mlp.usable(net, x):
            assert rows % 8
            continue
        y = mfma_mlp.mlp_apply(net, x)
        grads = torch.autograd.grad(y, list(net.parameters()), g)
        rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-12))  # noqa: E731
        assert rel(y, y_ref) < 2e-2, rel(y, y_ref)
        for (name, _), a, b in zip(net.named_parameters(), grads, grads_ref):
            assert a.shape == b.shape, name
            assert rel(a, b) < 2e-2, (name, rel(a, b))
        with torch.inference_mode():  # rollout path: no saved activations
            y2 = mfma_mlp.mlp_apply(net, x)
        assert torch.equal(y2, y.detach())  # row results independent of train/eval path


def test_mfma_twin_mlps_match_single_launches():
    """Actor + critic through shared launches == each net alone (bitwise), grads too."""
    from rsl_rl.modules import mfma_mlp
    from rsl_rl.modules.actor_critic import mlp, get_activation
    torch.manual_seed(1)
    a = mlp(48, [512, 256, 128], 12, get_activation("elu")).cuda()
    c = mlp(50, [512, 256, 128], 1, get_activation("elu")).cuda()
    xa, xc = torch.randn(8192, 48, device="cuda"), torch.randn(8192, 50, device="cuda")
    ya, yc = mfma_mlp.mlps_apply([a, c], [xa, xc])
    ga = torch.randn_like(ya)
    gc = torch.randn_like(yc)
    g2 = torch.autograd.grad((ya * ga).sum() + (yc * gc).sum(), list(a.parameters()) + list(c.parameters()))
    ya1 = mfma_mlp.mlp_apply(a, xa)
    yc1 = mfma_mlp.mlp_apply(c, xc)
    g1 = torch.autograd.grad((ya1 * ga).sum() + (yc1 * gc).sum(), list(a.parameters()) + list(c.parameters()))
    assert torch.equal(ya, ya1) and torch.equal(yc, yc1)
    for u, v in zip(g2, g1):
        assert torch.equal(u, v)


@pytest.mark.parametrize("clipped", [True, False])
def test_fused_ppo_loss_matches_reference_loss(clipped):
    """mfma_mlp.ppo_loss (fused kernels) vs rsl_rl's torch statement of the loss:
    value, statistics, KL and the gradients w.r.t. mean, std and value."""
    from torch.distributions import Normal
    from rsl_rl.modules import mfma_mlp
    torch.manual_seed(0)
    M, A, clip, vcoef, ecoef = 24576, 12, 0.2, 1.0, 0.01
    mu = torch.randn(M, A, device="cuda", requires_grad=True)
    std = (0.5 + torch.rand(A, device="cuda")).requires_grad_()
    value = torch.randn(M, 1, device="cuda", requires_grad=True)
    actions = mu.detach() + 0.3 * torch.randn(M, A, device="cuda")
    old_mu = mu.detach() + 0.05 * torch.randn(M, A, device="cuda")
    old_sigma = (std.detach() * (1 + 0.1 * torch.rand(M, A, device="cuda")))
    old_logp = Normal(old_mu, old_sigma).log_prob(actions).sum(-1, keepdim=True)
    adv, ret = torch.randn(M, 1, device="cuda"), torch.randn(M, 1, device="cuda")
    target = value.detach() + 0.3 * torch.randn(M, 1, device="cuda")  # some rows clip, some do not

    # torch statement (rsl_rl v1.0.2 PPO.update)
    d = Normal(mu, mu * 0.0 + std)
    ratio = torch.exp(d.log_prob(actions).sum(-1) - torch.squeeze(old_logp))
    s1 = -torch.squeeze(adv) * ratio
    s2 = -torch.squeeze(adv) * torch.clamp(ratio, 1 - clip, 1 + clip)
    surr = torch.max(s1, s2).mean()
    if clipped:
        vc = target + (value - target).clamp(-clip, clip)
        vl = torch.max((value - ret).pow(2), (vc - ret).pow(2)).mean()
    else:
        vl = (ret - value).pow(2).mean()
    loss_ref = surr + vcoef * vl - ecoef * d.entropy().sum(-1).mean()
    sig = mu.detach() * 0 + std.detach()
    kl_ref = torch.sum(torch.log(sig / old_sigma + 1.0e-5) + (old_sigma ** 2 + (old_mu - mu.detach()) ** 2)
                       / (2.0 * sig ** 2) - 0.5, axis=-1).mean()
    g_ref = torch.autograd.grad(loss_ref, (mu, std, value))

    loss, stats = mfma_mlp.ppo_loss(mu, std, value, actions, old_logp, old_mu, old_sigma, adv, ret, target, clip,
                                    clipped, vcoef, ecoef)
    g = torch.autograd.grad(loss, (mu, std, value))
    close = lambda a, b, tol: abs(float(a) - float(b)) <= tol * (abs(float(b)) + 1e-6)  # noqa: E731
    assert close(loss, loss_ref, 1e-4) and close(stats[0], surr, 1e-4) and close(stats[1], vl, 1e-4)
    assert close(stats[2], kl_ref, 1e-4)
    for a, b in zip(g, g_ref):
        assert a.shape == b.shape
        assert float((a - b).norm() / (b.norm() + 1e-12)) < 1e-4


@pytest.mark.parametrize("n", [512, 4])
def test_rollout_graph_matches_eager_rollouts(tmp_path, n):
    """OnPolicyRunner's captured collection loop (_RolloutGraph) replays the same
    rollouts as the eager loop: same env states, storage, policy and logged
    episode statistics (rewbuffer/lenbuffer/ep_infos) after several iterations.
    4 envs is BASELINE configs[0]'s size (seed 1, legged_robot_config.py:245): 24-row
    mini-batches through the fused update."""
    import json
    from legged_gym.utils.helpers import class_to_dict
    from rsl_rl.runners import OnPolicyRunner
    out = {}
    for graph in (False, True):
        env = make("go2", n, env__episode_length_s=0.5)  # 25-step episodes: resets inside every rollout
        _, train_cfg = task_registry.get_cfgs("go2")
        cfg = class_to_dict(train_cfg)
        cfg["runner"]["rollout_graph"] = graph
        torch.manual_seed(0)
        torch.cuda.manual_seed(0)
        log_dir = tmp_path / f"graph{int(graph)}"
        runner = OnPolicyRunner(env, cfg, log_dir=str(log_dir), device="cuda:0")
        runner.learn(4, init_at_random_ep_len=True)
        torch.cuda.synchronize()
        runner.writer.flush()
        st = runner.alg.storage
        scal = [json.loads(line) for line in open(log_dir / "scalars.jsonl")]
        out[graph] = dict(
            root=env.root_states.clone(), obs=env.obs_buf.clone(), step=env.common_step_counter,
            dev_step=int(env._d_step_counter), st_obs=st.observations.clone(), st_act=st.actions.clone(),
            st_rew=st.rewards.clone(), st_done=st.dones.clone(),
            params=[p.detach().clone() for p in runner.alg.actor_critic.parameters()],
            scalars={(s["tag"], s["step"]): s["value"] for s in scal
                     if not s["tag"].startswith("Perf") and "time" not in s["tag"]})
        env.close()
    e, g = out[False], out[True]
    assert e["step"] == g["step"] == g["dev_step"] == e["dev_step"] == 4 * cfg["runner"]["num_steps_per_env"] + 1
    for k in ("root", "obs", "st_obs", "st_act", "st_rew", "st_done"):
        assert torch.equal(e[k], g[k]), k
    for a, b in zip(e["params"], g["params"]):
        assert torch.equal(a, b)
    assert e["scalars"].keys() == g["scalars"].keys()
    assert any(k[0] == "Train/mean_reward" for k in e["scalars"])
    for k, v in e["scalars"].items():
        assert v == pytest.approx(g["scalars"][k], rel=1e-6, abs=1e-7), k


@pytest.mark.parametrize("task", ["go2", "h1"])
def test_name_queries_match_the_model(task):
    """The C ABI's name queries return the URDF body/DOF names in the simulator's order, and
    find_body resolves the env's feet / contact indices (find_actor_rigid_body_handle)."""
    import isaacgym  # noqa: F401
    from legged_gym.envs import task_registry
    from legged_gym.utils import get_args
    env, _ = task_registry.make_env(name=task, args=get_args(["--task", task, "--num_envs", "8", "--headless"]))
    assert env.sim.body_names() == list(env.model.body_names)
    assert env.sim.dof_names() == list(env.model.dof_names)
    for i in env.feet_indices.tolist():
        assert env.sim.find_body(env.model.body_names[i]) == i
    assert env.sim.find_body("no_such_link") == -1
    assert env.sim.find_dof(env.model.dof_names[-1]) == len(env.model.dof_names) - 1
    lib = env.sim.lib
    assert lib.lgs_get_body_name(env.sim.handle, len(env.model.body_names)) is None


def test_humanoid_feet_state_is_the_feet_rows_after_each_step():
    """h1_env.py:48-56's feet_state / feet_pos / feet_vel: the feet rows of the rigid body
    states after the step (gathered when read, no launch per step), and a task's own
    assignment is kept."""
    env = make("h1", 64)
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(3):
        env.step(0.3 * torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g))
        rows = env.rigid_body_states_view[:, env.feet_indices, :]
        assert env.feet_state.shape == (env.num_envs, len(env.feet_indices), 13)
        assert torch.equal(env.feet_state, rows)
        assert torch.equal(env.feet_pos, rows[:, :, :3]) and torch.equal(env.feet_vel, rows[:, :, 7:10])
    own = torch.zeros(3)
    env.feet_pos = own
    assert env.feet_pos is own
