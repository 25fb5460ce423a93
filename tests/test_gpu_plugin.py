"""Task plugin API: a task registered with task_registry.register may add
reward terms as Python ``_reward_<name>`` methods (legged_robot.py:817-840 looks them up by
name), and reset_idx may be called on any subset of envs (:723).  A Python copy of a native
term must give the native term's rewards, sums and extras."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.envs.base.legged_robot import LeggedRobot  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402


class Go2WithPythonTerms(LeggedRobot):
    """Go2 whose lin_vel_z and feet_air_time terms are Python methods (the reference's own
    formulas, legged_robot.py:843-845, 912-923) instead of kernel terms."""

    def _reward_lin_vel_z_py(self):
        return torch.square(self.base_lin_vel[:, 2])

    def _reward_action_rate_py(self):
        return torch.sum(torch.square(self.last_actions - self.actions), dim=1)


def _make(name, cls, edit):
    env_cfg, train_cfg = task_registry.get_cfgs("go2")
    cfg = copy.deepcopy(env_cfg)
    edit(cfg)
    task_registry.register(name, cls, cfg, copy.deepcopy(train_cfg))
    args = get_args(["--task", name, "--num_envs", "256", "--headless"])
    env, _ = task_registry.make_env(name=name, args=args)
    return env


def test_python_reward_terms_match_native_terms():
    def native(cfg):
        pass

    def python(cfg):
        cfg.rewards.scales.lin_vel_z_py = cfg.rewards.scales.lin_vel_z
        cfg.rewards.scales.action_rate_py = cfg.rewards.scales.action_rate
        cfg.rewards.scales.lin_vel_z = 0.0
        cfg.rewards.scales.action_rate = 0.0

    envs = [_make("go2_native", LeggedRobot, native), _make("go2_pyterms", Go2WithPythonTerms, python)]
    nat, py = envs
    assert not nat._py_rewards and [n for n, _ in py._py_rewards] == ["action_rate_py", "lin_vel_z_py"]
    assert py.task_params.defer_reward_total == 1 and py.task_params.num_extra_sums == 2
    for e in envs:
        e.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    rename = {"lin_vel_z": "lin_vel_z_py", "action_rate": "action_rate_py"}
    for step in range(60):
        a = 0.6 * torch.randn(256, 12, device="cuda", generator=g)
        if step == 30:  # a batch of time-outs: resets, extras
            for e in envs:
                e.episode_length_buf = torch.full_like(e.episode_length_buf, int(e.max_episode_length))
        outs = [e.step(a) for e in envs]
        (o1, _, r1, d1, x1), (o2, _, r2, d2, x2) = outs
        assert torch.equal(o1, o2) and torch.equal(d1, d2)  # the state never depends on the rewards
        # only the summation order of the terms differs (native terms first, then Python ones)
        torch.testing.assert_close(r2, r1, rtol=1e-5, atol=1e-6)
        for k in nat._sum_names:
            torch.testing.assert_close(py.episode_sums[rename.get(k, k)], nat.episode_sums[k], rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(x2["episode"]["rew_" + rename.get(k, k)], x1["episode"]["rew_" + k],
                                       rtol=1e-4, atol=1e-7)
    assert d1.any()


def test_reset_idx_subset_through_the_python_api():
    env = _make("go2_subset", LeggedRobot, lambda cfg: None)
    env.reset()
    for _ in range(20):
        env.step(0.5 * torch.randn(256, 12, device="cuda"))
    ids = torch.tensor([3, 17, 200], device="cuda")
    sums = env._episode_sums[:, ids].clone()
    keep = torch.ones(256, dtype=torch.bool, device="cuda")
    keep[ids] = False
    root_keep = env.root_states[keep].clone()
    env.reset_idx(ids)
    assert (env.episode_length_buf[ids] == 0).all() and (env.actions[ids] == 0).all()
    assert env.reset_buf[ids].all()
    assert torch.equal(env.root_states[keep], root_keep)
    assert (env._episode_sums[:, ids] == 0).all()
    want = (sums.mean(dim=1) / env.max_episode_length_s).cpu().numpy()
    got = np.array([float(env.extras["episode"]["rew_" + k]) for k in env._sum_names])
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)
    env.step(torch.zeros(256, 12, device="cuda"))  # the env keeps stepping normally


def _extra_term(k):
    def term(self):
        return (k + 1) * torch.square(self.base_lin_vel[:, 2]) + 0.01 * k
    return term


Go2ManyTerms = type("Go2ManyTerms", (LeggedRobot,),
                    {f"_reward_extra_{k:02d}": _extra_term(k) for k in range(26)})


def test_many_python_reward_terms_on_two_envs_per_wave():
    """Go2 runs two envs per wave (32 lanes per env): with 10 native + 26 Python terms the
    episode-sum rows (36) exceed the lanes of one env, and every row must still join the
    reset-time extras and be zeroed on reset (post_physics strides the rows)."""
    def edit(cfg):
        for k in range(26):
            setattr(cfg.rewards.scales, f"extra_{k:02d}", 0.1)
    env = _make("go2_many_terms", Go2ManyTerms, edit)
    assert env.task_params.num_extra_sums == 26
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(10):
        env.step(0.5 * torch.randn(256, 12, device="cuda", generator=g))
    names = list(env._sum_names)
    assert len(names) >= 36
    before = {k: env.episode_sums[k].clone() for k in names}
    # a whole batch of time-outs: every env resets at the next step
    env.episode_length_buf = torch.full_like(env.episode_length_buf, int(env.max_episode_length))
    _, _, _, _, extras = env.step(0.5 * torch.randn(256, 12, device="cuda", generator=g))
    assert env.reset_buf.all()
    for k in names:
        # the resetting step adds its own term, hands the sums to the extras, then zeroes them
        assert (env.episode_sums[k] == 0).all(), k
        if k.startswith("extra_"):  # positive terms: a row left out of the extras would read 0
            assert float(extras["episode"]["rew_" + k]) > float(before[k].mean()) / env.max_episode_length_s * 0.99, k


from legged_gym.envs.h1.h1_env import H1Robot  # noqa: E402


class H1WithKneeTerm(H1Robot):
    """An H1 task with a Python reward that reads non-foot rigid-body rows (the knees and the
    pelvis), as a reference-style task written against refreshed body states would."""

    def _reward_knee_height(self):
        self.seen_body_states = self.rigid_body_states_view.clone()
        knees = [i for i, n in enumerate(self.body_names) if "knee" in n]
        return self.rigid_body_states_view[:, knees, 2].mean(dim=1) - self.rigid_body_states_view[:, 0, 2]


def test_python_reward_reads_every_body_row_equal_to_the_oracle():
    """With a Python reward term the step refreshes EVERY rigid_body_states row (not only the
    feet), on the pre-reset state the reference's compute_reward sees; the rows the term read
    equal the CPU oracle's forward kinematics of that step, bit for bit."""
    import bridge
    env_cfg, train_cfg = task_registry.get_cfgs("h1")
    cfg = copy.deepcopy(env_cfg)
    cfg.rewards.scales.knee_height = 0.5
    task_registry.register("h1_knee_term", H1WithKneeTerm, cfg, copy.deepcopy(train_cfg))
    env, _ = task_registry.make_env(name="h1_knee_term", args=get_args(["--task", "h1_knee_term", "--num_envs", "64",
                                                                        "--headless"]))
    assert env.task_params.body_state_mask == 0 and env.task_params.write_body_states == 1
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(8):
        env.step(0.4 * torch.randn(64, env.num_actions, device="cuda", generator=g))
    snap = bridge.snapshot(env)
    a = 0.4 * torch.randn(64, env.num_actions, device="cuda", generator=g)
    ref = bridge.step(env, snap, a.cpu().numpy(), env.common_step_counter)
    env.step(a)
    torch.cuda.synchronize()
    B = env.num_bodies
    want = ref["rbs"].reshape(64, B, 13)
    seen = env.seen_body_states.cpu().numpy()
    np.testing.assert_array_equal(seen, want)
    np.testing.assert_array_equal(env.rigid_body_states.view(64, B, 13).cpu().numpy(), want)
    knees = [i for i, n in enumerate(env.body_names) if "knee" in n]
    assert len(knees) == 2 and not (seen[:, knees, 2] == 0).all()
