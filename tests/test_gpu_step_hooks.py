"""A task's Python per-step hooks.

The reference's humanoid tasks override ``_post_physics_step_callback`` (the gait phase,
h1_env.py:55-65, g1_env.py:56-105) and ``compute_observations`` (h1_env.py:68-95,
g1_env.py:108-141); a task may override ``check_termination`` the same way.  The step then
runs its split path (``LeggedRobot._split_post_physics``): the native launches of
post_physics_step with the task's Python code at the reference's points between them.  Each
test below registers a subclass whose hook is this build's own torch statement of what the
kernel computes and checks it against the native task on the same seeds and actions: the
state never depends on the hooks, so the two envs stay in lock-step.
"""
import copy
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.envs.h1.h1_env import H1Robot  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402

N = 64


def _pair(name, cls, edit=lambda cfg: None, task="h1"):
    """The native task and `cls` registered on the same (edited) cfg, same seed."""
    env_cfg, train_cfg = task_registry.get_cfgs(task)
    cfg = copy.deepcopy(env_cfg)
    cfg.noise.add_noise = False
    edit(cfg)
    envs = []
    for nm, c in ((name + "_native", task_registry.get_task_class(task)), (name, cls)):
        task_registry.register(nm, c, copy.deepcopy(cfg), copy.deepcopy(train_cfg))
        env, _ = task_registry.make_env(name=nm, args=get_args(["--task", nm, "--num_envs", str(N), "--headless"]))
        env.reset()
        envs.append(env)
    return envs


def _steps(envs, n, seed, scale=0.5, check=None):
    g = torch.Generator(device="cuda").manual_seed(seed)
    dones = 0
    for t in range(n):
        if t == n // 2:  # a batch of time-outs halfway: resets, extras
            for e in envs:
                e.episode_length_buf = torch.full_like(e.episode_length_buf, int(e.max_episode_length))
        a = scale * torch.randn(N, envs[0].num_actions, device="cuda", generator=g)
        outs = [e.step(a) for e in envs]
        dones += int(outs[0][3].sum())
        if check is not None:
            check(t, outs)
    assert dones > 0
    return outs


class H1PyObs(H1Robot):
    """compute_observations as torch ops on the env's buffers (the humanoid layout: angular
    velocity, gravity, commands, joint offsets and velocities, actions, sin/cos of the gait
    phase; privileged = base linear velocity + the same)."""

    def compute_observations(self):
        s = self.obs_scales
        ang = 2.0 * math.pi * self.phase
        body = [self.base_ang_vel * s.ang_vel, self.projected_gravity, self.commands[:, :3] * self.commands_scale,
                (self.dof_pos - self.default_dof_pos) * s.dof_pos, self.dof_vel * s.dof_vel, self.actions,
                torch.sin(ang)[:, None], torch.cos(ang)[:, None]]
        self.obs_buf = torch.cat(body, dim=-1)
        self.privileged_obs_buf = torch.cat([self.base_lin_vel * s.lin_vel] + body, dim=-1)
        if self.add_noise:
            self.obs_buf += (2 * torch.rand_like(self.obs_buf) - 1) * self.noise_scale_vec
        self.calls = getattr(self, "calls", 0) + 1


def test_python_compute_observations_equals_the_kernel_observation():
    nat, py = _pair("h1_pyobs", H1PyObs)
    assert py._hooks == {"compute_observations"} and py._split_step and not nat._split_step
    py.calls = 0  # (BaseTask.reset stepped once)

    def check(t, outs):
        (o1, p1, r1, d1, _), (o2, p2, r2, d2, _) = outs
        assert torch.equal(d1, d2)
        torch.testing.assert_close(o2, o1, rtol=0, atol=1e-6)
        torch.testing.assert_close(p2, p1, rtol=0, atol=1e-6)
        torch.testing.assert_close(r2, r1, rtol=1e-6, atol=1e-7)
        assert o2.data_ptr() == py._obs_bufs[py._buf_idx].data_ptr()  # returned in the env's buffers
    _steps([nat, py], 40, 0, check=check)
    assert py.calls == 40


class H1PyPhase(H1Robot):
    """_post_physics_step_callback computing the gait phase in torch, reference style: fresh
    phase / leg_phase tensors every step, the feet refreshed first, then super()."""

    def _post_physics_step_callback(self):
        self.update_feet_state()
        period, offset = 0.8, 0.5
        # (fmod: exact, like the remainder of the reference's `%` on these positive times)
        self.phase = torch.fmod(self.episode_length_buf * self.dt, period) / period
        self.leg_phase = torch.stack([self.phase, torch.fmod(self.phase + offset, 1.0)], dim=-1)
        self.seen_feet_z = self.feet_pos[:, :, 2].clone()
        return super()._post_physics_step_callback()


def test_python_callback_gait_phase_drives_the_kernel_rewards_and_obs():
    nat, py = _pair("h1_pyphase", H1PyPhase)
    assert py._hooks == {"_post_physics_step_callback"}
    phase_buf = py._bound["phase"]

    def check(t, outs):
        (o1, p1, r1, d1, _), (o2, p2, r2, d2, _) = outs
        assert torch.equal(d1, d2)
        # copied into the kernel's buffer, then read back by its rewards and observations
        assert py.phase is phase_buf
        assert torch.equal(py.phase, nat.phase) and torch.equal(py.leg_phase, nat.leg_phase)
        assert torch.equal(o2, o1) and torch.equal(p2, p1)
        assert torch.equal(r2, r1)
        # the callback saw this step's feet rows (before the reset of the step)
        assert py.seen_feet_z.shape == (N, 2) and bool((py.seen_feet_z != 0).any())
    _steps([nat, py], 40, 1, check=check)


class H1PyTermination(H1Robot):
    """check_termination restated in torch (contact on a termination body, roll / pitch
    limits, time-outs), plus `extra_height`: a base below it also terminates."""
    extra_height = None

    def check_termination(self):
        f = torch.norm(self.contact_forces[:, self.termination_contact_indices, :], dim=-1)
        self.reset_buf = torch.any(f > 1.0, dim=1)
        self.reset_buf |= torch.logical_or(torch.abs(self.rpy[:, 1]) > 1.0, torch.abs(self.rpy[:, 0]) > 0.8)
        if self.extra_height is not None:
            self.reset_buf |= self.root_states[:, 2] < self.extra_height
        self.time_out_buf = self.episode_length_buf > self.max_episode_length
        self.reset_buf |= self.time_out_buf


def test_python_check_termination_decides_the_resets():
    nat, py = _pair("h1_pyterm", H1PyTermination)
    assert py._hooks == {"check_termination"} and py.task_params.defer_reward_total == 1

    def check(t, outs):
        (o1, p1, r1, d1, x1), (o2, p2, r2, d2, x2) = outs
        assert torch.equal(d2, d1) and torch.equal(x2["time_outs"], x1["time_outs"])
        assert torch.equal(o2, o1)
        torch.testing.assert_close(r2, r1, rtol=1e-6, atol=1e-7)
    _steps([nat, py], 40, 2, check=check)
    # a termination of the task's own: every env whose base is below 2 m resets at once
    py.extra_height = 2.0
    a = torch.zeros(N, py.num_actions, device="cuda")
    _, _, _, d, _ = py.step(a)
    assert bool(d.all()) and bool((py.episode_length_buf == 0).all())


class H1RefFeet(H1Robot):
    """The reference's _init_foot body (h1_env.py:34-42: acquire + wrap the rigid body state,
    feet rows copied by advanced indexing) and no callback override."""

    def _init_foot(self):
        from isaacgym import gymtorch
        self.feet_num = len(self.feet_indices)
        rbs = self.gym.acquire_rigid_body_state_tensor(self.sim)
        self.rigid_body_states = gymtorch.wrap_tensor(rbs)
        self.rigid_body_states_view = self.rigid_body_states.view(self.num_envs, -1, 13)
        self.feet_state = self.rigid_body_states_view[:, self.feet_indices, :]
        self.feet_pos = self.feet_state[:, :, :3]
        self.feet_vel = self.feet_state[:, :, 7:10]


def test_task_feet_copies_are_refreshed_every_step():
    env_cfg, train_cfg = task_registry.get_cfgs("h1")
    task_registry.register("h1_ref_feet", H1RefFeet, copy.deepcopy(env_cfg), copy.deepcopy(train_cfg))
    env, _ = task_registry.make_env(name="h1_ref_feet", args=get_args(["--task", "h1_ref_feet", "--num_envs", str(N),
                                                                        "--headless"]))
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    first = None
    for t in range(12):
        env.step(0.5 * torch.randn(N, env.num_actions, device="cuda", generator=g))
        rows = env.rigid_body_states.view(N, -1, 13)[:, env.feet_indices, :]
        assert torch.equal(env.feet_state, rows)
        assert torch.equal(env.feet_pos, rows[:, :, :3]) and torch.equal(env.feet_vel, rows[:, :, 7:10])
        if first is None:
            first = env.feet_pos.clone()
    assert not torch.equal(env.feet_pos, first)  # not frozen at the first step's copy


class H1HookCounter(H1PyPhase):
    """H1PyPhase plus a device-side count of the callback's executions (an in-place add,
    so a captured rollout replays it)."""

    def _post_physics_step_callback(self):
        if not hasattr(self, "hook_steps"):
            self.hook_steps = torch.zeros((), dtype=torch.int64, device=self.device)
        self.hook_steps += 1
        return super()._post_physics_step_callback()


class H1HostSyncHook(H1PyPhase):
    """A callback the collection graph cannot capture: the reference's resampling idiom,
    env ids through .nonzero() (legged_robot.py:492-494), reads the device from the host."""

    def _post_physics_step_callback(self):
        ids = (self.episode_length_buf % 50 == 0).nonzero(as_tuple=False).flatten()
        self.resample_count = int(ids.numel())
        return super()._post_physics_step_callback()


def _runner(name, cls, rollout_graph=True):
    env_cfg, train_cfg = task_registry.get_cfgs("h1")
    env_cfg, train_cfg = copy.deepcopy(env_cfg), copy.deepcopy(train_cfg)
    train_cfg.runner.rollout_graph = rollout_graph
    task_registry.register(name, cls, env_cfg, train_cfg)
    args = get_args(["--task", name, "--num_envs", str(N), "--headless"])
    env, _ = task_registry.make_env(name=name, args=args)
    runner, _ = task_registry.make_alg_runner(env=env, name=name, args=args, log_root=None)
    return env, runner


def test_runner_captures_and_replays_the_python_hooks():
    env, runner = _runner("h1_hook_graph", H1HookCounter)
    c0, h0 = env.common_step_counter, int(env.hook_steps)
    runner.learn(3)  # eager, then captured and replayed twice
    assert runner._rollout_graph is not None
    torch.cuda.synchronize()
    assert env.common_step_counter - c0 == 3 * runner.num_steps_per_env
    assert int(env.hook_steps) - h0 == 3 * runner.num_steps_per_env  # the hook ran inside every replay


def test_runner_collects_eagerly_when_a_hook_cannot_be_captured():
    """The failed capture leaves no trace: the run equals one that never tried (same seeds)."""
    with pytest.warns(UserWarning, match="collecting eagerly"):
        env_a, ra = _runner("h1_hostsync_try", H1HostSyncHook)
        ra.learn(3)
    assert ra._rollout_graph is None and ra._rollout_graph_failed
    env_b, rb = _runner("h1_hostsync_eager", H1HostSyncHook, rollout_graph=False)
    rb.learn(3)
    torch.cuda.synchronize()
    assert env_a.common_step_counter == env_b.common_step_counter
    for pa, pb in zip(ra.alg.actor_critic.parameters(), rb.alg.actor_critic.parameters()):
        assert torch.equal(pa, pb)
    for k in ("rewards", "actions", "values", "dones"):
        assert torch.equal(getattr(ra.alg.storage, k), getattr(rb.alg.storage, k))
