"""LeggedRobot on the MI355X-native simulator.

Drop-in for the reference's ``legged_gym/envs/base/legged_robot.py`` (class
``LeggedRobot``, :21-941): same constructor signature, same VecEnv attributes
and buffers, same cfg semantics.  The difference is where the work happens:

* ``step()`` (:615-647) is ONE launch of ``lgs_step`` — PD torques, the
  decimation physics substeps and the whole ``post_physics_step`` (:673-709:
  commands, termination, rewards, reset, push, observations) run in a HIP
  kernel with one wavefront per env.  There are no per-term PyTorch ops and no
  device->host syncs (the reference's ``nonzero()`` at :511, :545, :697 are
  in-kernel masks).
* ``create_sim`` builds the articulated model from the URDF (IsaacGym asset
  semantics, :294-407) and hands it to ``libleggedsim``.

Buffers that the caller keeps across a step (obs, privileged obs, resets,
time-outs) are double-buffered, because the reference returns fresh tensors
each step and rsl_rl holds references to them across the next ``step()``.
"""
import os
import time

import numpy as np
import torch

from isaacgym.torch_utils import get_axis_params, to_torch, torch_rand_float
from legged_gym import LEGGED_GYM_ROOT_DIR
from legged_gym.envs.base.base_task import BaseTask
from legged_gym.utils.helpers import class_to_dict
from leggedsim import cabi, native
from leggedsim.model import load_model
from leggedsim.selfcollision import build_self_collision
from leggedsim.task import build_task_params
from legged_gym.utils.terrain import Terrain

from .env_spec import derive_env_spec
from .legged_robot_config import LeggedRobotCfg


class _GymTensorAPI:
    """The gym tensor refreshes a task's own methods call (legged_robot.py:639, 678-679;
    h1_env.py:37, 49).  The step writes the bound tensors in place, so the refreshes are
    no-ops, except the rigid body states: the step refreshes only the rows the task reads
    (lgs_task_params.body_state_mask: the humanoids' feet), and
    refresh_rigid_body_state_tensor refreshes every body (lgs_forward_kinematics)."""

    def __init__(self, env):
        self._env = env

    def refresh_dof_state_tensor(self, sim):
        pass

    def refresh_actor_root_state_tensor(self, sim):
        pass

    def refresh_net_contact_force_tensor(self, sim):
        pass

    def refresh_rigid_body_state_tensor(self, sim):
        self._env._sync_stream()
        self._env.sim.forward_kinematics()

    # acquire_*_tensor (legged_robot.py:83-86, h1_env.py:37): the bound state tensors
    # themselves (gymtorch.wrap_tensor returns its argument), so a task's own _init_foot
    # written against gym gets views of the live state
    def acquire_actor_root_state_tensor(self, sim):
        return self._env.root_states

    def acquire_dof_state_tensor(self, sim):
        return self._env.dof_state

    def acquire_net_contact_force_tensor(self, sim):
        return self._env._contact_forces

    def acquire_rigid_body_state_tensor(self, sim):
        return self._env.rigid_body_states


class _DeferredExtras:
    """The extras of a control step issued by lgs_step_deferred, left to the step's consumer
    (include/leggedsim.h).  `fields` are include/ppo_mlp.h pmlp_env_extras' values, for the
    rollout's next policy launch to do the work in; run() issues lgs_step_extras instead.
    Whoever issues the work sets `consumed` (a host flag: a captured rollout replays the
    consumer's launch on the device without it)."""

    def __init__(self, env, E, k):
        self.env, self.k = env, k
        self.E = cabi.EnvBuffers.from_buffer_copy(E)  # this step's pointers (the struct is reused two steps on)
        if getattr(env, "_push_state", None) is None:
            env._push_state = env.sim.push_state()
        vsim, pushed = env._push_state
        tp = env.task_params
        self.fields = dict(acc=E.episode_acc, acc_next=E.episode_acc_next,
                           nsum=tp.num_rewards + (1 if tp.has_termination_reward else 0) + tp.num_extra_sums,
                           ep_len_s=float(tp.max_episode_length_s), ep_means=E.ep_means, ep_snapshot=E.ep_snapshot,
                           time_out=E.time_out, carry=E.time_outs_carry, last_root_vel=E.last_root_vel, vsim=vsim,
                           pushed=pushed, push=int(bool(tp.push_robots)), step_counter=E.step_counter)
        self.consumed = False

    def run(self):
        """The work on its own launch (what lgs_step issues after the step)."""
        if not self.consumed:
            self.consumed = True
            self.env.sim.step_extras(self.E, self.k)


class LeggedRobot(BaseTask):
    obs_layout = cabi.OBS_QUADRUPED
    # rigid_body_states rows each step refreshes: "feet" (all the reference's humanoid envs
    # read, h1_env.py:34-52) or "all"; None = "all" when the task has Python `_reward_*` terms
    # (they may read any body row, as after the reference's per-step refresh, h1_env.py:48-56),
    # else "feet".  self.gym.refresh_rigid_body_state_tensor always refreshes every body.
    rigid_body_state_bodies = None
    hip_dof_indices = ()
    max_contacts = 8
    max_rows = 32
    max_self_contacts = 4  # contact slots self contacts may take per substep (cfg.asset.self_collisions == 0)
    # The reference's per-step methods a task may override in Python, as its H1Robot / G1Robot
    # do (h1_env.py:55-95, g1_env.py:56-141): the step then takes its split path and calls the
    # override at the reference's point of post_physics_step (:692, :695, :704), between native
    # launches (_split_post_physics).  _get_noise_scale_vec may be overridden too: its vector is
    # the one the kernel's observation noise uses (leggedsim/task.py).
    PYTHON_STEP_HOOKS = ("_post_physics_step_callback", "check_termination", "compute_observations")
    # The per-step methods that stay inside the kernel (legged_robot.py:649-671, 519-555,
    # 557-594, 770-787, 673-709): _compute_torques runs in the substep loop, the rest inside
    # the reset / push / reward stages of the same launch.  The kernel never calls a Python
    # method there, so an override would train as if it had not: construction refuses it.
    # Python `_reward_<name>` terms ARE supported (_prepare_reward_function).
    NATIVE_STEP_METHODS = ("_compute_torques", "_resample_commands", "_push_robots", "compute_reward",
                           "post_physics_step", "_reset_dofs", "_reset_root_states")
    # env buffers the kernel reads after _post_physics_step_callback: a callback that rebinds
    # one (the reference's assigns fresh phase / leg_phase tensors) is copied into it
    CALLBACK_BUFFERS = ("commands", "phase", "leg_phase", "base_lin_vel", "base_ang_vel", "projected_gravity", "rpy")

    def __init__(self, cfg: LeggedRobotCfg, sim_params, physics_engine, sim_device, headless):
        self._refuse_native_step_overrides()
        self._hooks = self.python_step_hooks()
        self.cfg = cfg
        self.sim_params = sim_params
        self.gym = _GymTensorAPI(self)
        self.height_samples = None
        self.debug_viz = False
        self.init_done = False
        self._parse_cfg(self.cfg)
        super().__init__(self.cfg, sim_params, physics_engine, sim_device, headless)
        self._init_buffers()
        self._prepare_reward_function()
        self._build_task()
        self.init_done = True

    @classmethod
    def _overridden(cls, names):
        """(name, owner) of each of `names` a task class defines outside the build's own classes."""
        from .humanoid import HumanoidRobot
        native = (BaseTask, LeggedRobot, HumanoidRobot)
        out = []
        for name in names:
            owner = next((k for k in cls.__mro__ if name in vars(k)), None)
            if owner is not None and owner not in native:
                out.append((name, owner))
        return out

    @classmethod
    def python_step_hooks(cls):
        """The PYTHON_STEP_HOOKS this task class overrides (the step's split path calls them)."""
        return frozenset(name for name, _ in cls._overridden(cls.PYTHON_STEP_HOOKS))

    @classmethod
    def _refuse_native_step_overrides(cls):
        bad = [f"{owner.__module__}.{owner.__qualname__}.{name}" for name, owner in cls._overridden(cls.NATIVE_STEP_METHODS)]
        if bad:
            raise NotImplementedError(
                f"{cls.__name__} overrides {', '.join(bad)}: the native step (one lgs_step launch) computes "
                "torques, command resampling, pushes, rewards and resets in a HIP kernel and never calls these "
                "methods, so the override would be silently ignored.  Supported plugin points: cfg values, "
                "Python `_reward_<name>` terms (scaled like the reference's), overrides of "
                f"{', '.join(cls.PYTHON_STEP_HOOKS)} and _get_noise_scale_vec, and reset_idx(env_ids); "
                "see INTEGRATION.md.")

    # ------------------------------------------------------------ config ----
    def _parse_cfg(self, cfg):
        """legged_robot.py:52-67"""
        self.dt = self.cfg.control.decimation * self.sim_params.dt
        self.obs_scales = self.cfg.normalization.obs_scales
        self.reward_scales = class_to_dict(self.cfg.rewards.scales)
        self.command_ranges = class_to_dict(self.cfg.commands.ranges)
        self.max_episode_length_s = self.cfg.env.episode_length_s
        self.max_episode_length = np.ceil(self.max_episode_length_s / self.dt)
        self.cfg.domain_rand.push_interval = np.ceil(self.cfg.domain_rand.push_interval_s / self.dt)

    # ------------------------------------------------------------- sim ------
    def create_sim(self):
        """Model + native sim creation (legged_robot.py:223-242, 281-407, 412-483)."""
        self.up_axis_idx = 2
        asset_path = self.cfg.asset.file.format(LEGGED_GYM_ROOT_DIR=LEGGED_GYM_ROOT_DIR)
        if not os.path.exists(asset_path) and os.environ.get("LEGGED_GYM_RESOURCES"):
            rel = asset_path.split("resources/", 1)[-1]
            asset_path = os.path.join(os.environ["LEGGED_GYM_RESOURCES"], rel)
        model = load_model(asset_path, collapse_fixed_joints=self.cfg.asset.collapse_fixed_joints)
        model_feet = {model.body_names.index(n) for n in model.body_names if self.cfg.asset.foot_name in n}
        model.reorder_points(model_feet)
        self.model = model
        spec = derive_env_spec(self.cfg, model, self.sim_params.dt, self.obs_layout, self.hip_dof_indices)
        self.spec = spec
        dev = self.device
        self.num_dof = spec.num_dof
        self.num_bodies = spec.num_bodies
        self.dof_names = spec.dof_names
        self.num_dofs = len(self.dof_names)
        self.body_names = spec.body_names
        self.feet_indices = torch.tensor(spec.feet_indices, dtype=torch.long, device=dev)
        self.penalised_contact_indices = torch.tensor(spec.penalised_contact_indices, dtype=torch.long, device=dev)
        self.termination_contact_indices = torch.tensor(spec.termination_contact_indices, dtype=torch.long, device=dev)
        self.base_init_state = torch.tensor(spec.base_init_state, device=dev)
        # rough terrain (utils/terrain.py): the height map the contact kernel samples
        self.terrain = None
        if self.cfg.terrain.mesh_type in ("heightfield", "trimesh"):
            self.terrain = Terrain(self.cfg.terrain, self.num_envs)
        self._get_env_origins()
        self.dof_pos_limits = torch.tensor(spec.dof_pos_limits, device=dev)
        self.dof_vel_limits = torch.tensor(spec.dof_vel_limits, device=dev)
        self.torque_limits = torch.tensor(spec.torque_limits, device=dev)

        # shape friction buckets (_process_rigid_shape_props, :429-439): torch CPU RNG as the reference
        friction = np.full(self.num_envs, self.cfg.terrain.static_friction, dtype=np.float32)
        if self.cfg.domain_rand.randomize_friction:
            fr = self.cfg.domain_rand.friction_range
            bucket_ids = torch.randint(0, 64, (self.num_envs, 1))
            buckets = torch_rand_float(fr[0], fr[1], (64, 1), device="cpu")
            self.friction_coeffs = buckets[bucket_ids]
            friction = self.friction_coeffs.view(-1).numpy().astype(np.float32)
        # base mass (_process_rigid_body_props, :480-482)
        added_mass = np.zeros(self.num_envs, dtype=np.float32)
        if self.cfg.domain_rand.randomize_base_mass:
            rng = self.cfg.domain_rand.added_mass_range
            added_mass = np.array([np.random.uniform(rng[0], rng[1]) for _ in range(self.num_envs)], dtype=np.float32)
        self.added_base_mass = added_mass

        sp = cabi.sim_params_from_cfg(self.cfg.sim, self.cfg.asset, max_contacts=self.max_contacts,
                                      max_rows=self.max_rows, ground_friction=float(self.cfg.terrain.static_friction))
        self._lgs_params = sp
        self.sim = native.Sim(model, sp, self.num_envs, self.sim_device_id)
        # names and body handles through the simulator, as the reference asks gym for them
        # (get_asset_rigid_body_names / get_asset_dof_names :342-343, find_actor_rigid_body_handle :388-407)
        self.body_names, self.dof_names = self.sim.body_names(), self.sim.dof_names()
        for attr in ("feet_indices", "penalised_contact_indices", "termination_contact_indices"):
            idx = getattr(self, attr)
            found = [self.sim.find_body(spec.body_names[int(i)]) for i in idx.tolist()]
            if found != idx.tolist():
                raise RuntimeError(f"{attr}: simulator body handles {found} != model indices {idx.tolist()}")
        self.sim.set_env_properties(friction, added_mass)
        self.shape_friction = friction
        # create_actor(..., self_collisions, 0) (:373-374): 0 lets the links of one robot collide
        self.self_collision = None
        if int(getattr(self.cfg.asset, "self_collisions", 1)) == 0:
            self.self_collision = build_self_collision(model, np.asarray(spec.default_dof_pos).reshape(-1),
                                                       max_self_contacts=self.max_self_contacts)
            self.sim.set_self_collision(self.self_collision)
        if self.terrain is not None:
            self._create_heightfield()
        else:
            self._create_ground_plane()

    def _create_ground_plane(self):
        """The plane is the z = 0 half-space inside the contact kernel (legged_robot.py:244-256)."""
        self.sim.set_heightfield(None, 0.0, 0.0, 0.0)

    def _create_heightfield(self):
        """gym.add_heightfield of legged_gym's rough-terrain path: the int16 map of
        utils/terrain.py, offset by -border_size in x and y."""
        tc = self.cfg.terrain
        self.sim.set_heightfield(self.terrain.heightsamples, tc.horizontal_scale, tc.vertical_scale, tc.border_size)
        self.height_samples = torch.tensor(self.terrain.heightsamples).view(
            self.terrain.tot_rows, self.terrain.tot_cols).to(self.device)

    def _get_env_origins(self):
        """Env origins (legged_robot.py:258-272): the terrain tiles on rough terrain
        (levels U{0..max_init_terrain_level}, types by env id, as legged_gym's
        rough-terrain path), otherwise a grid."""
        if self.terrain is not None:
            tc = self.cfg.terrain
            self.custom_origins = True
            self.env_origins = torch.zeros(self.num_envs, 3, device=self.device, requires_grad=False)
            max_init_level = tc.max_init_terrain_level if tc.curriculum else tc.num_rows - 1
            max_init_level = min(max_init_level, tc.num_rows - 1)  # a level must be a terrain row
            self.terrain_levels = torch.randint(0, max_init_level + 1, (self.num_envs,), device=self.device)
            self.terrain_types = torch.div(torch.arange(self.num_envs, device=self.device),
                                           (self.num_envs / tc.num_cols), rounding_mode="floor").to(torch.long)
            self.max_terrain_level = tc.num_rows
            self.terrain_origins = torch.from_numpy(self.terrain.env_origins).to(self.device).to(torch.float)
            self.env_origins[:] = self.terrain_origins[self.terrain_levels, self.terrain_types]
            return
        self.custom_origins = False
        self.env_origins = torch.zeros(self.num_envs, 3, device=self.device, requires_grad=False)
        num_cols = np.floor(np.sqrt(self.num_envs))
        num_rows = np.ceil(self.num_envs / num_cols)
        xx, yy = torch.meshgrid(torch.arange(num_rows), torch.arange(num_cols), indexing="ij")
        spacing = self.cfg.env.env_spacing
        self.env_origins[:, 0] = spacing * xx.flatten()[: self.num_envs]
        self.env_origins[:, 1] = spacing * yy.flatten()[: self.num_envs]
        self.env_origins[:, 2] = 0.0

    # --------------------------------------------------------- buffers ------
    def _init_buffers(self):
        """State tensors bound to the simulator + the env's working buffers (:69-186)."""
        N, D, B, dev = self.num_envs, self.num_dof, self.num_bodies, self.device
        self.root_states = torch.zeros(N, 13, dtype=torch.float, device=dev)
        self.dof_state = torch.zeros(N * D, 2, dtype=torch.float, device=dev)
        self._contact_forces = torch.zeros(N * B, 3, dtype=torch.float, device=dev)
        self.rigid_body_states = torch.zeros(N * B, 13, dtype=torch.float, device=dev)
        # initial placement: base_init_state at the origin with +-1 m xy jitter (:364-370)
        self.root_states[:] = self.base_init_state
        self.root_states[:, :3] += self.env_origins
        self.root_states[:, :2] += torch_rand_float(-1.0, 1.0, (N, 2), device=dev)
        self.dof_pos = self.dof_state.view(N, D, 2)[..., 0]
        self.dof_vel = self.dof_state.view(N, D, 2)[..., 1]
        self.base_quat = self.root_states[:, 3:7]
        self.base_pos = self.root_states[:N, 0:3]
        self.contact_forces = self._contact_forces.view(N, -1, 3)
        self.rigid_body_states_view = self.rigid_body_states.view(N, -1, 13)
        self.sim.bind(self.root_states, self.dof_state, self._contact_forces, self.rigid_body_states)
        self._stream = None
        self._sync_stream()
        self.defer_extras = False  # OnPolicyRunner sets it around its collection loop (step())
        self._deferred = None

        self.common_step_counter = 0
        self.extras = {}
        self.gravity_vec = to_torch(get_axis_params(-1.0, self.up_axis_idx), device=dev).repeat((N, 1))
        self.forward_vec = to_torch([1.0, 0.0, 0.0], device=dev).repeat((N, 1))
        self.torques = torch.zeros(N, self.num_actions, dtype=torch.float, device=dev)
        self.p_gains = torch.zeros(self.num_actions, dtype=torch.float, device=dev)
        self.d_gains = torch.zeros(self.num_actions, dtype=torch.float, device=dev)
        self.actions = torch.zeros(N, self.num_actions, dtype=torch.float, device=dev)
        self.last_actions = torch.zeros(N, self.num_actions, dtype=torch.float, device=dev)
        self.last_dof_vel = torch.zeros(N, D, dtype=torch.float, device=dev)
        self.last_root_vel = torch.zeros(N, 6, dtype=torch.float, device=dev)
        self.commands = torch.zeros(N, self.cfg.commands.num_commands, dtype=torch.float, device=dev)
        if self.commands.shape[1] != 4:
            raise ValueError("the native step expects commands.num_commands == 4")
        self.commands_scale = torch.tensor([self.obs_scales.lin_vel, self.obs_scales.lin_vel, self.obs_scales.ang_vel],
                                           device=dev)
        nf = len(self.feet_indices)
        self.feet_air_time = torch.zeros(N, nf, dtype=torch.float, device=dev)
        self.last_contacts = torch.zeros(N, nf, dtype=torch.bool, device=dev)
        self.base_lin_vel = torch.zeros(N, 3, dtype=torch.float, device=dev)
        self.base_ang_vel = torch.zeros(N, 3, dtype=torch.float, device=dev)
        self.projected_gravity = torch.zeros(N, 3, dtype=torch.float, device=dev)
        self.rpy = torch.zeros(N, 3, dtype=torch.float, device=dev)
        self._episode_length = torch.zeros(N, dtype=torch.long, device=dev)
        self.phase = torch.zeros(N, dtype=torch.float, device=dev)
        self.leg_phase = torch.zeros(N, 2, dtype=torch.float, device=dev)
        # double-buffered step outputs
        P = self.num_privileged_obs
        self._obs_bufs = [torch.zeros(N, self.num_obs, dtype=torch.float, device=dev) for _ in range(2)]
        self._priv_bufs = [torch.zeros(N, P, dtype=torch.float, device=dev) for _ in range(2)] if P else [None, None]
        self._reset_bufs = [torch.ones(N, dtype=torch.bool, device=dev) for _ in range(2)]
        self._timeout_bufs = [torch.zeros(N, dtype=torch.bool, device=dev) for _ in range(2)]
        self._buf_idx = 0
        self.obs_buf = self._obs_bufs[0]
        self.privileged_obs_buf = self._priv_bufs[0]
        self.reset_buf = torch.ones(N, dtype=torch.long, device=dev)  # long at init, bool after a step (base_task.py:43)
        self.time_out_buf = self._timeout_bufs[0]
        self.rew_buf = torch.zeros(N, dtype=torch.float, device=dev)
        self.noise_scale_vec = self._get_noise_scale_vec(self.cfg)

        # default joint angles and PD gains by name substring, last match wins (:168-186)
        self.default_dof_pos = torch.tensor(self.spec.default_dof_pos, device=dev)
        self.p_gains[:] = torch.tensor(self.spec.p_gains, device=dev)
        self.d_gains[:] = torch.tensor(self.spec.d_gains, device=dev)
        self.dof_pos[:] = self.default_dof_pos

    @property
    def episode_length_buf(self):
        return self._episode_length

    @episode_length_buf.setter
    def episode_length_buf(self, value):
        # rsl_rl rebinds this attribute (randint_like) before learning; keep the
        # kernel's buffer and copy the values in.
        self._episode_length.copy_(value.to(device=self.device, dtype=torch.long))

    def _get_noise_scale_vec(self, cfg):
        """legged_robot.py:188-219 (quadruped) / h1_env.py:10-31 (humanoid layout).  A task's
        override returns the vector the kernel's observation noise then uses (task params)."""
        self.add_noise = self.cfg.noise.add_noise
        return torch.tensor(self.spec.noise_scale_vec, device=self.device)

    # ------------------------------------------- per-step Python hooks -----
    # The native step has done each of these when a task override runs (the override's
    # super() call therefore adds nothing): the split path (_split_post_physics) calls the
    # override at the reference's point of post_physics_step.
    def _post_physics_step_callback(self):
        """legged_robot.py:488-517: command resampling and heading (and the humanoid gait
        phase, h1_env.py:55-65) are computed by lgs_post_physics_prepare before an override runs."""

    def check_termination(self):
        """legged_robot.py:711-721: reset_buf / time_out_buf hold the kernel's termination when
        an override runs; whatever the override leaves in them decides the resets."""

    def compute_observations(self):
        """legged_robot.py:789-811: obs_buf / privileged_obs_buf hold the kernel's observations
        (noise added) when an override runs; what it leaves there is clipped and returned."""

    def _refresh_task_views(self):
        """Per-step refresh of tensors a task derived from the state (HumanoidRobot: feet)."""

    def _prepare_reward_function(self):
        """Drop zero scales, multiply the rest by dt; dict order = alphabetical (:817-840).

        Terms the kernel knows run inside the fused step.  A term it does not know is looked
        up as ``self._reward_<name>`` like the reference does (a task subclass may define it);
        such Python terms run between the two halves of the post-physics stack, on the same
        pre-reset state the reference's compute_reward sees (step() then takes the split path:
        lgs_step_physics, lgs_post_physics_rewards, the Python terms, lgs_post_physics_finish)."""
        self.reward_scales = dict(self.spec.reward_scales)
        self.reward_names = list(self.spec.reward_names)
        self._native_reward_names, self._py_rewards = [], []
        for n in self.reward_names:
            if cabi.REWARD_ALIASES.get(n, n) in cabi.REWARD_ID:
                self._native_reward_names.append(n)
            else:  # AttributeError like the reference's getattr (:834) when the task has no such method
                self._py_rewards.append((n, getattr(self, "_reward_" + n)))
        py_names = [n for n, _ in self._py_rewards]
        self._sum_names = [n for n in self.spec.sum_names if n not in py_names] + py_names
        nsum = len(self._sum_names)
        self._episode_sums = torch.zeros(nsum, self.num_envs, dtype=torch.float, device=self.device)
        self.episode_sums = {name: self._episode_sums[i] for i, name in enumerate(self._sum_names)}
        # two accumulator slots, one per env-buffer parity: a deferred step's consumer zeroes the
        # next step's slot while its workgroups still read this step's (lgs_step_deferred)
        self._episode_acc = torch.zeros(2, nsum + 1, dtype=torch.float, device=self.device)
        self._ep_means = torch.zeros(nsum, dtype=torch.float, device=self.device)
        self._time_outs = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)

    # ------------------------------------------------------ native task -----
    def _build_task(self):
        nvec = torch.as_tensor(self.noise_scale_vec).reshape(-1)
        if nvec.numel() != self.num_obs:
            raise ValueError(f"_get_noise_scale_vec returned {nvec.numel()} entries for {self.num_obs} observations")
        self.task_params = build_task_params(self)
        self.sim.set_task(self.task_params)
        self._env_structs = [self._make_env_struct(i) for i in range(2)]
        self._bound = {name: getattr(self, name) for name in self.CALLBACK_BUFFERS}
        self._split_step = bool(self._py_rewards or self._hooks)

    def _make_env_struct(self, i):
        E = cabi.EnvBuffers()
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        E.actions = p(self.actions)
        E.last_actions = p(self.last_actions)
        E.last_dof_vel = p(self.last_dof_vel)
        E.last_root_vel = p(self.last_root_vel)
        E.torques = p(self.torques)
        E.commands = p(self.commands)
        E.feet_air_time = p(self.feet_air_time)
        E.last_contacts = p(self.last_contacts)
        E.episode_length = p(self._episode_length)
        E.obs = p(self._obs_bufs[i])
        E.priv_obs = p(self._priv_bufs[i])
        E.rew = p(self.rew_buf)
        E.reset = p(self._reset_bufs[i])
        E.time_out = p(self._timeout_bufs[i])
        E.episode_sums = p(self._episode_sums)
        E.episode_acc = p(self._episode_acc[i])
        E.episode_acc_next = p(self._episode_acc[i ^ 1])
        E.base_lin_vel = p(self.base_lin_vel)
        E.base_ang_vel = p(self.base_ang_vel)
        E.projected_gravity = p(self.projected_gravity)
        E.rpy = p(self.rpy)
        E.env_origins = p(self.env_origins)
        E.phase = p(self.phase)
        E.leg_phase = p(self.leg_phase)
        E.rew_terms = None
        E.step_counter = p(self._d_step_counter)
        E.ep_means = p(self._ep_means)
        E.ep_snapshot = None  # set per step (step())
        E.time_outs_carry = p(self._time_outs) if self.cfg.env.send_timeouts else None
        return E

    @property
    def common_step_counter(self):
        """The reference's step counter (legged_robot.py:116).  The native step keys its
        Philox streams on a DEVICE copy that lgs_step advances itself, so a captured
        rollout graph draws new noise/commands on every replay; this host mirror counts
        eagerly issued steps plus those the runner reports via `account_replayed_steps`."""
        return self._step_mirror

    @common_step_counter.setter
    def common_step_counter(self, value):
        self._step_mirror = int(value)
        if getattr(self, "_d_step_counter", None) is None:
            self._d_step_counter = torch.zeros((), dtype=torch.int64, device=self.device)
        self._d_step_counter.fill_(self._step_mirror)

    def account_replayed_steps(self, n):
        """A graph replay of n captured steps advanced the device counter by n."""
        self._step_mirror += int(n)

    def _sync_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream:
            self.sim.set_stream(s)
            self._stream = s

    # ------------------------------------------------------------ step ------
    def step(self, actions):
        """Apply actions, simulate `decimation` substeps, post-physics; one launch (three
        launches and the Python terms when the task defines Python reward terms).

        With `defer_extras` set (OnPolicyRunner, around its collection loop) the step's extras
        launch is left to the step's consumer: infos["_deferred_extras"] describes it, and the
        rollout's next policy launch does that work on its own rows (pmlp_env_extras).  Until
        then extras["episode"] / extras["time_outs"] are the previous step's; a step nobody
        consumed is completed at the next step, reset_idx or flush_extras()."""
        self._sync_stream()
        self.flush_extras()
        self._buf_idx ^= 1
        i = self._buf_idx
        E = self._env_structs[i]
        # the kernel reads the caller's actions in place (clipped copy into self.actions);
        # anything else is copied first
        if (actions.is_cuda and actions.dtype == torch.float32 and actions.is_contiguous() and
                actions.shape == self.actions.shape and actions.device == self.actions.device):
            E.actions_in = actions.data_ptr()
        else:
            self.actions.copy_(actions)
            E.actions_in = None
        # this step's extras["episode"] values (a fresh buffer per step, like the
        # reference's per-reset tensors; inside a captured rollout, one per step)
        snap = torch.empty(len(self._sum_names), dtype=torch.float, device=self.device)
        E.ep_snapshot = snap.data_ptr()
        job = None
        if self._split_step:
            self._split_post_physics(E, i)
        elif self.defer_extras:
            self.sim.step_deferred(E, self._step_mirror)  # the extras: the consumer's (job)
            job = self._deferred = _DeferredExtras(self, E, self._step_mirror)
            self._refresh_task_views()
        else:
            self.sim.step(E, self._step_mirror)  # + extras, episode_acc reset, step counter
            self._refresh_task_views()
        self._step_mirror += 1
        if self.cfg.env.test:
            self._pace_to_real_time()
        self.obs_buf = self._obs_bufs[i]
        self.privileged_obs_buf = self._priv_bufs[i]
        self.reset_buf = self._reset_bufs[i]
        self.time_out_buf = self._timeout_bufs[i]
        self.extras["episode"] = {"rew_" + k: snap[j] for j, k in enumerate(self._sum_names)}
        if self.cfg.env.send_timeouts:
            self.extras["time_outs"] = self._time_outs
        if job is not None:
            self.extras["_deferred_extras"] = job
        else:
            self.extras.pop("_deferred_extras", None)
        return self.obs_buf, self.privileged_obs_buf, self.rew_buf, self.reset_buf, self.extras

    def flush_extras(self):
        """Complete a deferred step's extras that no consumer has taken (lgs_step_extras)."""
        job, self._deferred = self._deferred, None
        if job is not None:
            job.run()

    def _split_post_physics(self, E, i):
        """step() for a task with Python reward terms or step hooks: the native launches of
        post_physics_step (legged_robot.py:673-709) with the task's Python code between them, in
        the reference's order -- physics; base-frame state and the native callback
        (lgs_post_physics_prepare); the task's _post_physics_step_callback; termination and the
        native rewards (lgs_post_physics_term_rewards); the task's check_termination; the
        Python reward terms, only_positive_rewards and the termination term; reset, push,
        observations and bookkeeping (lgs_post_physics_finish); the task's compute_observations.
        Without a callback override the first two native parts are one launch
        (lgs_post_physics_rewards)."""
        k, hooks = self._step_mirror, self._hooks
        self.sim.step_physics(E, k)
        self.reset_buf, self.time_out_buf = self._reset_bufs[i], self._timeout_bufs[i]
        if "_post_physics_step_callback" in hooks:
            self.sim.post_physics_prepare(E, k)
            self._post_physics_step_callback()
            self._rebind(self.CALLBACK_BUFFERS)
            self.sim.post_physics_term_rewards(E, k)
        else:
            self.sim.post_physics_rewards(E, k)
            self._refresh_task_views()
        if "check_termination" in hooks:
            self.check_termination()
            # the reference's assigns fresh tensors (torch.any / a comparison): the kernel's
            # reset and time-out bytes take their values
            for name, buf in (("reset_buf", self._reset_bufs[i]), ("time_out_buf", self._timeout_bufs[i])):
                cur = getattr(self, name)
                if cur is not buf:
                    buf.copy_(cur.reshape(buf.shape))
                    setattr(self, name, buf)
        if self.task_params.defer_reward_total:
            self._python_rewards()
        self.sim.post_physics_finish(E, k)
        if "compute_observations" in hooks:
            self.obs_buf, self.privileged_obs_buf = self._obs_bufs[i], self._priv_bufs[i]
            self.compute_observations()
            clip = self.cfg.normalization.clip_observations  # step()'s clip (legged_robot.py:643-646)
            for name, buf in (("obs_buf", self._obs_bufs[i]), ("privileged_obs_buf", self._priv_bufs[i])):
                cur = getattr(self, name)
                if buf is None:
                    continue
                if cur is not buf:
                    buf.copy_(cur.reshape(buf.shape))
                buf.clamp_(-clip, clip)
                setattr(self, name, buf)

    def _rebind(self, names):
        """A hook that assigned a fresh tensor to a buffer the kernel reads: copy it in."""
        for name in names:
            bound, cur = self._bound[name], getattr(self, name)
            if cur is not bound:
                bound.copy_(cur.reshape(bound.shape))
                setattr(self, name, bound)

    def _pace_to_real_time(self):
        """cfg.env.test (play.py): simulated time does not run ahead of the wall clock
        (legged_robot.py:631-635: gym.get_sim_time vs gym.get_elapsed_time, both counted
        from the sim's creation).  Never inside a captured graph (nothing would wait)."""
        if torch.cuda.is_current_stream_capturing():
            return
        if getattr(self, "_wall_t0", None) is None:
            self._wall_t0, self._sim_time = time.perf_counter(), 0.0
        self._sim_time += self.dt
        ahead = self._sim_time - (time.perf_counter() - self._wall_t0)
        if ahead > 0:
            time.sleep(ahead)

    def _python_rewards(self):
        """compute_reward (legged_robot.py:770-787) for the Python terms: the kernel left the
        raw sum of its own terms in rew_buf (defer_reward_total); add these terms (scale
        already times dt), then the only_positive_rewards clip and the termination term."""
        nat = len(self._native_reward_names) + (1 if "termination" in self.reward_scales else 0)
        for k, (name, fn) in enumerate(self._py_rewards):
            rew = fn() * self.reward_scales[name]
            self.rew_buf += rew
            self._episode_sums[nat + k] += rew
        if self.cfg.rewards.only_positive_rewards:
            self.rew_buf[:] = torch.clip(self.rew_buf[:], min=0.0)
        if "termination" in self.reward_scales:
            rew = (self.reset_buf & ~self.time_out_buf).float() * self.reward_scales["termination"]
            self.rew_buf += rew
            self.episode_sums["termination"] += rew

    def reset_idx(self, env_ids):
        """reset_idx (legged_robot.py:723-768) for any subset of envs: one masked launch
        (lgs_reset_idx) resets dofs, root states and commands, zeroes the actions and
        buffers, sets reset_buf[env_ids] = 1 and fills extras["episode"] (means of the
        reset envs' episode sums / episode_length_s) and extras["time_outs"]."""
        if len(env_ids) == 0:
            return
        self._sync_stream()
        self.flush_extras()
        ids = torch.as_tensor(env_ids, device=self.device).long().view(-1)
        mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        mask[ids] = 1
        E = self._env_structs[self._buf_idx]
        snap = torch.empty(len(self._sum_names), dtype=torch.float, device=self.device)
        E.ep_snapshot = snap.data_ptr()
        self.sim.reset_idx(E, mask, self.common_step_counter)
        self.extras["episode"] = {"rew_" + k: snap[i] for i, k in enumerate(self._sum_names)}
        if self.cfg.env.send_timeouts:
            self.extras["time_outs"] = self._time_outs

    def post_physics_step(self):
        raise RuntimeError("post_physics_step runs inside the fused native step()")

    # -------------------------------------------------------- utilities -----
    def close(self):
        self.sim.close()
