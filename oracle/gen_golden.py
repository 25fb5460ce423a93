"""Generate golden vectors by running the REFERENCE's own Python post-physics stack.

Test infrastructure only (run here, in the container that has /root/reference;
the outputs are committed as small .npz fixtures under tests/golden/).

How: a throw-away shim directory provides the two missing dependencies the
reference imports: an ``isaacgym`` package whose ``torch_utils``
restates the helper functions legged_gym uses, and ``rsl_rl`` placeholders.
Then, per task, a duck-typed instance of the reference's env class
(``Cls.__new__`` + the attributes ``_init_buffers`` would create) runs its own
``_compute_torques`` and ``post_physics_step`` (legged_robot.py:649-709) on
seeded random post-physics states.  Physics itself (gym.simulate) is not run:
the state is the input.

Random draws: every ``torch_rand_float`` / ``torch.rand_like`` call of the
reference is answered with the build's Philox4x32-10 draws keyed exactly as
the HIP kernel keys them (env, step, stream, index), so reset / push / command
resampling / observation noise are comparable bit-for-bit in their inputs.

Usage:  python oracle/gen_golden.py [out_dir]
"""
import ctypes as C
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

TORCH_UTILS = r'''
import numpy as np
import torch

def to_torch(x, dtype=torch.float, device="cuda:0", requires_grad=False):
    return torch.tensor(x, dtype=dtype, device=device, requires_grad=requires_grad)

def get_axis_params(value, axis_idx, x_value=0.0, dtype=np.float64, n_dims=3):
    zs = np.zeros((n_dims,))
    zs[axis_idx] = 1.0
    params = np.where(zs == 1.0, value, zs)
    params[0] = x_value
    return list(params.astype(dtype))

def torch_rand_float(lower, upper, shape, device):
    return (upper - lower) * torch.rand(*shape, device=device) + lower

def normalize(x, eps: float = 1e-9):
    return x / x.norm(p=2, dim=-1).clamp(min=eps, max=None).unsqueeze(-1)

def quat_apply(a, b):
    shape = b.shape
    a = a.reshape(-1, 4)
    b = b.reshape(-1, 3)
    xyz = a[:, :3]
    t = xyz.cross(b, dim=-1) * 2
    return (b + a[:, 3:] * t + xyz.cross(t, dim=-1)).view(shape)

def quat_rotate_inverse(q, v):
    shape = q.shape
    q_w = q[:, -1]
    q_vec = q[:, :3]
    a = v * (2.0 * q_w ** 2 - 1.0).unsqueeze(-1)
    b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
    c = q_vec * torch.bmm(q_vec.view(shape[0], 1, 3), v.view(shape[0], 3, 1)).squeeze(-1) * 2.0
    return a - b + c
'''


def make_shims(d):
    os.makedirs(os.path.join(d, "isaacgym"))
    for name in ("__init__", "gymapi", "gymutil", "terrain_utils"):
        open(os.path.join(d, "isaacgym", name + ".py"), "w").write("")
    open(os.path.join(d, "isaacgym", "gymtorch.py"), "w").write(
        "def wrap_tensor(t):\n    return t\n\ndef unwrap_tensor(t):\n    return t\n")
    open(os.path.join(d, "isaacgym", "torch_utils.py"), "w").write(TORCH_UTILS)
    os.makedirs(os.path.join(d, "rsl_rl"))
    open(os.path.join(d, "rsl_rl", "__init__.py"), "w").write("")
    open(os.path.join(d, "rsl_rl", "env.py"), "w").write("class VecEnv:\n    pass\n")
    open(os.path.join(d, "rsl_rl", "runners.py"), "w").write("class OnPolicyRunner:\n    pass\n")


class FakeGym:
    """Records the sim-visible state written through set_*_tensor_indexed."""

    def __init__(self, env):
        self.env = env

    def refresh_dof_state_tensor(self, sim): pass
    def refresh_actor_root_state_tensor(self, sim): pass
    def refresh_net_contact_force_tensor(self, sim): pass
    def refresh_rigid_body_state_tensor(self, sim): pass

    def set_actor_root_state_tensor_indexed(self, sim, root, ids, n):
        ids = ids.long()
        self.env._sim_root[ids] = root[ids].clone()

    def set_dof_state_tensor_indexed(self, sim, dof, ids, n):
        ids = ids.long()
        D = self.env.num_dof
        v = dof.view(self.env.num_envs, D, 2)
        self.env._sim_dof.view(self.env.num_envs, D, 2)[ids] = v[ids].clone()


def main(out_dir):
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, os.path.join(HERE, "..", "unitree-rl-gym_amd"))
    from leggedsim import cabi
    from leggedsim.model import load_model
    lib = cabi.load_oracle()

    shim = tempfile.mkdtemp(prefix="lgs_shim_")
    make_shims(shim)
    sys.path.insert(0, REF)
    sys.path.insert(0, shim)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    import legged_gym.envs as ref_envs  # noqa: F401  (registers the reference tasks)
    from legged_gym.utils.task_registry import task_registry
    import legged_gym.envs.base.legged_robot as lr_mod

    seed = 1
    ctx = {"stream": None, "env_ids": None, "step": 0, "calls": 0}

    def philox(envs, stream, index):
        return np.array([lib.orc_uniform(seed, int(e), ctx["step"], stream, int(index)) for e in envs], np.float32)

    def rand_float(lower, upper, shape, device):
        rows, cols = shape
        envs = ctx["env_ids"] if ctx["env_ids"] is not None else np.arange(rows)
        stream = ctx["stream"]
        if stream in (cabi.STREAM_CMD, cabi.STREAM_RESET_CMD):
            u = philox(envs, stream, ctx["calls"])[:, None]
            ctx["calls"] += 1
        else:
            u = np.stack([philox(envs, stream, j) for j in range(cols)], axis=1)
        return (upper - lower) * torch.from_numpy(u) + lower

    lr_mod.torch_rand_float = rand_float
    Base = lr_mod.LeggedRobot
    orig = {n: getattr(Base, n) for n in ("_resample_commands", "_reset_dofs", "_reset_root_states", "_push_robots",
                                          "reset_idx")}

    def wrap_resample(self, env_ids):
        prev = ctx["stream"], ctx["env_ids"]
        ctx["stream"] = cabi.STREAM_RESET_CMD if ctx.get("in_reset") else cabi.STREAM_CMD
        ctx["env_ids"] = env_ids.cpu().numpy()
        ctx["calls"] = 0
        orig["_resample_commands"](self, env_ids)
        ctx["stream"], ctx["env_ids"] = prev

    def wrap_reset_dofs(self, env_ids):
        ctx["stream"], ctx["env_ids"] = cabi.STREAM_RESET_DOF, env_ids.cpu().numpy()
        orig["_reset_dofs"](self, env_ids)

    def wrap_reset_root(self, env_ids):
        ctx["stream"], ctx["env_ids"] = cabi.STREAM_RESET_ROOT, env_ids.cpu().numpy()
        orig["_reset_root_states"](self, env_ids)

    def wrap_push(self):
        ctx["stream"], ctx["env_ids"] = cabi.STREAM_PUSH, None
        orig["_push_robots"](self)

    def wrap_reset_idx(self, env_ids):
        ctx["in_reset"] = True
        orig["reset_idx"](self, env_ids)
        ctx["in_reset"] = False

    Base._resample_commands = wrap_resample
    Base._reset_dofs = wrap_reset_dofs
    Base._reset_root_states = wrap_reset_root
    Base._push_robots = wrap_push
    Base.reset_idx = wrap_reset_idx

    real_rand_like = torch.rand_like

    def rand_like(t):
        n, o = t.shape
        u = np.stack([philox(np.arange(n), cabi.STREAM_NOISE, k) for k in range(o)], axis=1)
        return torch.from_numpy(u)

    os.makedirs(out_dir, exist_ok=True)
    R = os.path.join(REF, "resources", "robots")
    tasks = {"go2": "go2/urdf/go2.urdf", "h1": "h1/urdf/h1.urdf", "g1": "g1_description/g1_12dof.urdf",
             "h1_2": "h1_2/h1_2_12dof.urdf"}
    for name, urdf in tasks.items():
        Cls = task_registry.task_classes[name]
        env_cfg, train_cfg = task_registry.get_cfgs(name)
        model = load_model(os.path.join(R, urdf))
        N, D, B = 64, model.num_dofs, model.num_bodies
        rng = np.random.default_rng(1234 + len(name))
        env = Cls.__new__(Cls)
        env.cfg = env_cfg
        env.sim_params = types.SimpleNamespace(dt=env_cfg.sim.dt)
        env.num_envs, env.num_dof, env.num_dofs, env.num_bodies = N, D, D, B
        env.num_obs = env_cfg.env.num_observations
        env.num_privileged_obs = env_cfg.env.num_privileged_obs
        env.num_actions = env_cfg.env.num_actions
        env.device = "cpu"
        env.headless = True
        env.viewer = None
        env.sim = None
        env.gym = FakeGym(env)
        env._parse_cfg(env_cfg)
        env.up_axis_idx = 2
        env.dof_names = list(model.dof_names)
        body_names = list(model.body_names)
        feet = [s for s in body_names if env_cfg.asset.foot_name in s]
        pen, term = [], []
        for k in env_cfg.asset.penalize_contacts_on:
            pen.extend([s for s in body_names if k in s])
        for k in env_cfg.asset.terminate_after_contacts_on:
            term.extend([s for s in body_names if k in s])
        env.feet_indices = torch.tensor([body_names.index(s) for s in feet], dtype=torch.long)
        env.penalised_contact_indices = torch.tensor([body_names.index(s) for s in pen], dtype=torch.long)
        env.termination_contact_indices = torch.tensor([body_names.index(s) for s in term], dtype=torch.long)
        # _process_dof_props (reference code path, :456-469)
        props = np.zeros(D, dtype=[("lower", np.float32), ("upper", np.float32), ("velocity", np.float32),
                                   ("effort", np.float32)])  # IsaacGym's dof-props structured array
        props["lower"], props["upper"] = model.dof_lower, model.dof_upper
        props["velocity"], props["effort"] = model.dof_velocity, model.dof_effort
        env._process_dof_props(props, 0)
        env.obs_buf = torch.zeros(N, env.num_obs)
        env.rew_buf = torch.zeros(N)
        env.reset_buf = torch.ones(N, dtype=torch.long)
        env.episode_length_buf = torch.zeros(N, dtype=torch.long)
        env.time_out_buf = torch.zeros(N, dtype=torch.bool)
        env.privileged_obs_buf = torch.zeros(N, env.num_privileged_obs) if env.num_privileged_obs else None
        env.base_init_state = torch.tensor(env_cfg.init_state.pos + env_cfg.init_state.rot +
                                           env_cfg.init_state.lin_vel + env_cfg.init_state.ang_vel, dtype=torch.float)
        env._get_env_origins()
        env.env_origins = env.env_origins.float()

        # ---- seeded post-physics state
        root = np.zeros((N, 13), np.float32)
        root[:, :3] = env.env_origins.numpy() + rng.normal(0, 0.3, (N, 3)).astype(np.float32)
        root[:, 2] = env_cfg.init_state.pos[2] * rng.uniform(0.6, 1.1, N)
        ax = rng.normal(size=(N, 3)); ax /= np.linalg.norm(ax, axis=1, keepdims=True)
        ang = rng.uniform(0, 0.5, N); ang[:6] = rng.uniform(0.9, 2.5, 6)   # some envs tilted past the limits
        yaw = rng.uniform(-np.pi, np.pi, N)
        q_tilt = np.concatenate([ax * np.sin(ang / 2)[:, None], np.cos(ang / 2)[:, None]], 1)
        q_yaw = np.stack([np.zeros(N), np.zeros(N), np.sin(yaw / 2), np.cos(yaw / 2)], 1)

        def qmul(a, b):
            x1, y1, z1, w1 = a.T
            x2, y2, z2, w2 = b.T
            return np.stack([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2, w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                             w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2, w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2], 1)
        root[:, 3:7] = qmul(q_yaw, q_tilt)
        root[:, 7:13] = rng.normal(0, 0.6, (N, 6))
        dof = np.zeros((N, D, 2), np.float32)
        dd = np.array([env_cfg.init_state.default_joint_angles[n] for n in env.dof_names], np.float32)
        dof[:, :, 0] = dd + rng.normal(0, 0.3, (N, D))
        dof[:, :, 1] = rng.normal(0, 2.0, (N, D))
        cf = np.zeros((N, B, 3), np.float32)
        fidx = env.feet_indices.numpy()
        cf[:, fidx, :] = rng.normal(0, 20, (N, len(fidx), 3))
        cf[:, fidx, 2] = np.abs(cf[:, fidx, 2]) * (rng.uniform(size=(N, len(fidx))) > 0.4)
        pidx = env.penalised_contact_indices.numpy()
        mask = rng.uniform(size=(N, len(pidx))) > 0.85
        cf[:, pidx, :] += (rng.normal(0, 2, (N, len(pidx), 3)) * mask[..., None]).astype(np.float32)
        tidx = env.termination_contact_indices.numpy()
        cf[6:9, tidx, 2] = 5.0                          # base/pelvis contacts -> termination
        rbs = np.zeros((N, B, 13), np.float32)
        rbs[:, :, :3] = rng.normal(0, 0.2, (N, B, 3)); rbs[:, :, 2] = np.abs(rbs[:, :, 2])
        rbs[:, :, 6] = 1.0
        rbs[:, :, 7:13] = rng.normal(0, 0.5, (N, B, 6))
        ep = rng.integers(0, 990, N).astype(np.int64)
        ep[10:13] = 499; ep[13:15] = 999; ep[15:18] = 1000  # resample boundaries, time-outs
        ep[18] = int(env_cfg.domain_rand.push_interval) - 1  # push boundary
        actions = rng.normal(0, 1.0, (N, D)).astype(np.float32); actions[0, 0] = 150.0  # clip path
        last_actions = rng.normal(0, 1.0, (N, D)).astype(np.float32)
        last_dof_vel = rng.normal(0, 2.0, (N, D)).astype(np.float32)
        commands = rng.uniform(-1, 1, (N, 4)).astype(np.float32); commands[:, 3] *= 3.14
        commands[20:23, :2] = 0.05  # zero-command branch
        air = rng.uniform(0, 0.8, (N, len(fidx))).astype(np.float32); air[:, 0] *= rng.uniform(size=N) > 0.3
        last_c = rng.uniform(size=(N, len(fidx))) > 0.5
        torques = rng.normal(0, 10.0, (N, D)).astype(np.float32)
        step_counter = 77

        # ---- reference: _compute_torques on the pre-step dof state (PD law, :649-671)
        env.dof_state = torch.from_numpy(dof.reshape(N * D, 2).copy())
        env.dof_pos = env.dof_state.view(N, D, 2)[..., 0]
        env.dof_vel = env.dof_state.view(N, D, 2)[..., 1]
        env.default_dof_pos = torch.tensor(dd).unsqueeze(0)
        env.p_gains = torch.zeros(D); env.d_gains = torch.zeros(D)
        for i, n in enumerate(env.dof_names):
            for k in env_cfg.control.stiffness.keys():
                if k in n:
                    env.p_gains[i] = env_cfg.control.stiffness[k]
                    env.d_gains[i] = env_cfg.control.damping[k]
        env.last_dof_vel = torch.from_numpy(last_dof_vel.copy())
        clipped = torch.clip(torch.from_numpy(actions), -env_cfg.normalization.clip_actions,
                             env_cfg.normalization.clip_actions)
        ref_torques = env._compute_torques(clipped).numpy().copy()

        # ---- reference: the buffers _init_buffers would create
        env.root_states = torch.from_numpy(root.copy())
        env.base_quat = env.root_states[:, 3:7]
        env.base_pos = env.root_states[:N, 0:3]
        from legged_gym.utils.isaacgym_utils import get_euler_xyz
        env.rpy = get_euler_xyz(env.base_quat)
        env.contact_forces = torch.from_numpy(cf.copy())
        env.common_step_counter = step_counter
        env.extras = {}
        env.noise_scale_vec = env._get_noise_scale_vec(env_cfg)
        env.gravity_vec = torch.tensor([[0.0, 0.0, -1.0]]).repeat(N, 1)
        env.forward_vec = torch.tensor([[1.0, 0.0, 0.0]]).repeat(N, 1)
        env.torques = torch.from_numpy(torques.copy())
        env.actions = clipped.clone()
        env.last_actions = torch.from_numpy(last_actions.copy())
        env.last_root_vel = torch.zeros(N, 6)
        env.commands = torch.from_numpy(commands.copy())
        env.commands_scale = torch.tensor([env.obs_scales.lin_vel, env.obs_scales.lin_vel, env.obs_scales.ang_vel])
        env.feet_air_time = torch.from_numpy(air.copy())
        env.last_contacts = torch.from_numpy(last_c.copy())
        env.base_lin_vel = torch.zeros(N, 3); env.base_ang_vel = torch.zeros(N, 3); env.projected_gravity = torch.zeros(N, 3)
        env.episode_length_buf = torch.from_numpy(ep.copy())
        if hasattr(env, "_init_foot"):
            env.feet_num = len(env.feet_indices)
            env.rigid_body_states = torch.from_numpy(rbs.reshape(N * B, 13).copy())
            env.rigid_body_states_view = env.rigid_body_states.view(N, -1, 13)
            env.feet_state = env.rigid_body_states_view[:, env.feet_indices, :]
            env.feet_pos = env.feet_state[:, :, :3]
            env.feet_vel = env.feet_state[:, :, 7:10]
        env._prepare_reward_function()
        env._sim_root = env.root_states.clone()
        env._sim_dof = env.dof_state.clone()
        torch.rand_like = rand_like
        ctx["step"] = step_counter
        try:
            env.post_physics_step()
        finally:
            torch.rand_like = real_rand_like
        # obs / priv clip of LeggedRobot.step (:643-646)
        clip = env_cfg.normalization.clip_observations
        obs = torch.clip(env.obs_buf, -clip, clip).numpy()
        priv = torch.clip(env.privileged_obs_buf, -clip, clip).numpy() if env.privileged_obs_buf is not None else np.zeros((N, 0), np.float32)
        nsum = len(env.episode_sums)
        extras_ep = np.array([env.extras["episode"]["rew_" + k].item() for k in env.episode_sums], np.float32) \
            if "episode" in env.extras else np.zeros(nsum, np.float32)
        out = dict(
            # inputs
            in_root=root, in_dof=dof.reshape(N * D, 2), in_cforce=cf, in_rbs=rbs, in_episode_length=ep,
            in_actions=actions, in_last_actions=last_actions, in_last_dof_vel=last_dof_vel, in_commands=commands,
            in_feet_air_time=air, in_last_contacts=last_c.astype(np.uint8), in_torques=torques,
            step_counter=np.array(step_counter), seed=np.array(seed),
            # reference-derived constants
            ref_p_gains=env.p_gains.numpy(), ref_d_gains=env.d_gains.numpy(),
            ref_default_dof_pos=env.default_dof_pos.numpy(), ref_dof_pos_limits=env.dof_pos_limits.numpy(),
            ref_noise_vec=env.noise_scale_vec.numpy(), ref_feet_indices=env.feet_indices.numpy(),
            ref_penalised=env.penalised_contact_indices.numpy(), ref_termination=env.termination_contact_indices.numpy(),
            ref_reward_names=np.array(list(env.reward_scales.keys())),
            ref_reward_scales=np.array([env.reward_scales[k] for k in env.reward_scales], np.float64),
            # outputs
            out_torques=ref_torques, out_obs=obs, out_priv=priv, out_rew=env.rew_buf.numpy(),
            out_reset=env.reset_buf.numpy().astype(np.uint8), out_time_out=env.time_out_buf.numpy().astype(np.uint8),
            out_root=env._sim_root.numpy(), out_dof=env._sim_dof.numpy(), out_commands=env.commands.numpy(),
            out_feet_air_time=env.feet_air_time.numpy(), out_last_contacts=env.last_contacts.numpy().astype(np.uint8),
            out_episode_length=env.episode_length_buf.numpy(),
            out_episode_sums=np.stack([env.episode_sums[k].numpy() for k in env.episode_sums]),
            out_extras_episode=extras_ep,
            out_last_actions=env.last_actions.numpy(), out_last_dof_vel=env.last_dof_vel.numpy(),
            # last_root_vel = the root_states TENSOR's velocities (:709): at a push step its xy
            # holds the all-env draw of _push_robots (:549-550), not the simulated state
            out_last_root_vel=env.last_root_vel.numpy(), out_root_tensor=env.root_states.numpy(),
            out_base_lin_vel=env.base_lin_vel.numpy(), out_base_ang_vel=env.base_ang_vel.numpy(),
            out_projected_gravity=env.projected_gravity.numpy(), out_rpy=env.rpy.numpy(),
        )
        path = os.path.join(out_dir, f"post_physics_{name}.npz")
        np.savez_compressed(path, **out)
        print(f"{name}: N={N} resets={int(env.reset_buf.sum())} timeouts={int(env.time_out_buf.sum())} -> {path}")

    # The recurrent-policy fixtures (tests/golden/lstm_policy_*.npz: the weights and 20-step
    # outputs of deploy/pre_train/*/motion.pt) are not regenerated here.  They were extracted
    # in round 1 with a loader that runs the archive's serialized code; the committed files
    # hold arrays only and are read with np.load(allow_pickle=False).  They are pinned without
    # executing anything from the archive: oracle/check_lstm_fixtures.py compares every
    # parameter, byte for byte, with the archive's raw tensor storages (zip entries), and the
    # outputs are re-derived from those weights with torch's nn.LSTM by tests/test_rsl_rl.py
    # (CPU) and tests/test_gpu_recurrent.py (the HIP LSTM kernels).

if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "tests", "golden"))
