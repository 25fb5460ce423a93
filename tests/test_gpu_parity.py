"""Bit-level parity of the HIP env step with the CPU oracle, through the C ABI.

The HIP kernel and the oracle are built without FP contraction and share their
transcendentals (csrc/lgs_detmath.h); every other operation runs in the same
order on both sides, and the constraint matrix A = Y Y^T is an fp32 fma chain on
both (v_mfma_f32_32x32x2_f32 is one, MI355X_MICROARCH.md).  So the bar here is
EXACT equality, for every env, of every state and output buffer:

* the post-physics half alone (lgs_post_physics) on the reference-generated golden
  inputs (tests/golden/post_physics_*.npz, made by the reference's own Python code)
  vs the golden outputs (1e-5, the reference's fp32 op order differs from ours) and
  vs the oracle on the same inputs (exact);
* the post-physics half on the HIP physics half's OWN output state vs the oracle's
  post-physics on that same state (exact): physics cannot mask an obs/reward error;
* the fused step == physics half + post half (exact);
* the fused step from identical states vs the oracle's fused step (exact), over
  several steps, all robots, ragged and full per-GPU env counts;
* reset_idx of a subset vs the oracle (exact) and the extras it reports.

The only quantity allowed to differ is the episode-extras accumulator (float
atomics over envs: the sum order is not fixed), compared at 1e-6 relative.
"""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
import bridge  # noqa: E402
from conftest import GOLDEN  # noqa: E402
from hostspec import host_buffers, make_spec  # noqa: E402
from leggedsim import cabi, native  # noqa: E402

TASKS = ["go2", "h1", "g1", "h1_2"]
STATE = ["root", "dofs", "cforce", "torques", "rbs"]
POST = ["obs", "priv_obs", "rew", "reset", "time_out", "commands", "episode_length", "feet_air_time",
        "last_contacts", "episode_sums", "last_actions", "last_dof_vel", "last_root_vel", "base_lin_vel",
        "base_ang_vel", "projected_gravity", "rpy", "phase", "leg_phase", "actions"]


def make(task, n, **edits):
    import copy
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env_cfg, _ = task_registry.get_cfgs(task)
    cfg = copy.deepcopy(env_cfg)
    for k, v in edits.items():
        sec, attr = k.split("__")
        setattr(getattr(cfg, sec), attr, v)
    env, _ = task_registry.make_env(name=task, args=args, env_cfg=cfg)
    return env


def env_arrays(env):
    """The env's buffers as host arrays, keyed like bridge.snapshot (the step just taken)."""
    torch.cuda.synchronize()
    t = lambda x: None if x is None else x.detach().cpu().numpy()  # noqa: E731
    return {"root": t(env.root_states), "dofs": t(env.dof_state), "cforce": t(env._contact_forces),
            "rbs": t(env.rigid_body_states), "torques": t(env.torques), "obs": t(env.obs_buf),
            "priv_obs": t(env.privileged_obs_buf), "rew": t(env.rew_buf), "reset": t(env.reset_buf).astype(np.uint8),
            "time_out": t(env.time_out_buf).astype(np.uint8), "commands": t(env.commands),
            "episode_length": t(env._episode_length), "feet_air_time": t(env.feet_air_time),
            "last_contacts": t(env.last_contacts).astype(np.uint8), "episode_sums": t(env._episode_sums),
            "last_actions": t(env.last_actions), "last_dof_vel": t(env.last_dof_vel),
            "last_root_vel": t(env.last_root_vel), "base_lin_vel": t(env.base_lin_vel),
            "base_ang_vel": t(env.base_ang_vel), "projected_gravity": t(env.projected_gravity), "rpy": t(env.rpy),
            "phase": t(env.phase), "leg_phase": t(env.leg_phase), "actions": t(env.actions)}


def per_env(a, n):
    if a.ndim >= 1 and a.shape[0] == n:
        return a.reshape(n, -1)
    if a.ndim == 2 and a.shape[1] == n:  # episode_sums [nsum, N]
        return a.T
    return a.reshape(n, -1)


def assert_exact(got, want, keys, n, what, skip_body_states=False):
    """Every env of every key bit-equal (+0 == -0); reports all mismatching keys first."""
    bad = []
    for k in keys:
        g, w = got.get(k), want.get(k)
        if g is None or w is None:
            continue
        if k == "rbs" and skip_body_states:
            continue
        g = per_env(np.asarray(g), n)
        w = per_env(np.asarray(w).reshape(np.asarray(got[k]).shape), n)
        assert np.isfinite(g.astype(np.float64)).all(), f"{what}: {k} not finite"
        diff = g != w
        if diff.any():
            envs = np.nonzero(diff.any(axis=1))[0]
            d = np.abs(g.astype(np.float64) - w.astype(np.float64)).max()
            bad.append(f"{k}: {len(envs)}/{n} envs differ (first env {envs[0]}, max |d| {d:.3e})")
    assert not bad, f"{what}: " + "; ".join(bad)


def writes_body_states(env):
    return bool(env.task_params.write_body_states)


# ------------------------------------------------------------------ golden --
def gpu_env_buffers(spec, N, golden):
    """Device buffers of a bare sim (no LeggedRobot) filled from a golden fixture."""
    b = host_buffers(spec, N)
    b["root"][:] = golden["in_root"]
    b["dofs"][:] = golden["in_dof"]
    b["cforce"][:] = golden["in_cforce"].reshape(-1, 3)
    b["rbs"][:] = golden["in_rbs"].reshape(-1, 13)
    b["actions"][:] = np.clip(golden["in_actions"], -100, 100)
    b["last_actions"][:] = golden["in_last_actions"]
    b["last_dof_vel"][:] = golden["in_last_dof_vel"]
    b["commands"][:] = golden["in_commands"]
    b["feet_air_time"][:] = golden["in_feet_air_time"]
    b["last_contacts"][:] = golden["in_last_contacts"]
    b["episode_length"][:] = golden["in_episode_length"]
    b["torques"][:] = golden["in_torques"]
    dev = {k: (None if v is None else torch.from_numpy(np.ascontiguousarray(v)).cuda()) for k, v in b.items()}
    return b, dev


def env_struct(dev):
    E = cabi.EnvBuffers()
    for k in bridge.ENV_KEYS:
        t = dev.get(k)
        setattr(E, k, None if t is None else t.data_ptr())
    E.rew_terms = None
    E.step_counter = None
    return E


@pytest.mark.parametrize("task", TASKS)
def test_post_physics_entry_matches_reference_golden(task):
    """lgs_post_physics on the reference-generated golden inputs == the reference's outputs
    (1e-5: the reference's torch op order) and == the oracle on the same inputs (exact)."""
    g = dict(np.load(f"{GOLDEN}/post_physics_{task}.npz"))
    spec = make_spec(task)
    N = g["in_actions"].shape[0]
    host, dev = gpu_env_buffers(spec, N, g)
    sim = native.Sim(spec.model, spec.sim_params, N, 0)
    sim.set_stream(torch.cuda.current_stream().cuda_stream)
    sim.bind(dev["root"], dev["dofs"], dev["cforce"], dev["rbs"])
    sim.set_task(spec.task)
    E = env_struct(dev)
    ep_means = torch.zeros(len(spec.sum_names), device="cuda")
    E.ep_means = ep_means.data_ptr()  # extras["episode"] of the step (k_step_extras)
    step = int(g["step_counter"])
    sim.post_physics(E, step)
    torch.cuda.synchronize()
    got = {k: (None if v is None else v.cpu().numpy()) for k, v in dev.items()}
    # the reference's own outputs: every env within 1e-5 (no env excluded)
    pairs = [("reset", "out_reset"), ("time_out", "out_time_out"), ("episode_length", "out_episode_length"),
             ("last_contacts", "out_last_contacts")]
    for k, r in pairs:
        np.testing.assert_array_equal(got[k], g[r], err_msg=k)
    close = [("base_lin_vel", "out_base_lin_vel"), ("base_ang_vel", "out_base_ang_vel"),
             ("projected_gravity", "out_projected_gravity"), ("rpy", "out_rpy"), ("commands", "out_commands"),
             ("rew", "out_rew"), ("episode_sums", "out_episode_sums"), ("feet_air_time", "out_feet_air_time"),
             ("root", "out_root"), ("dofs", "out_dof"), ("obs", "out_obs"), ("last_actions", "out_last_actions"),
             ("last_dof_vel", "out_last_dof_vel")]
    if spec.num_privileged_obs:
        close.append(("priv_obs", "out_priv"))
    for k, r in close:
        np.testing.assert_allclose(got[k], g[r], rtol=1e-5, atol=1e-5, err_msg=k)
    assert g["out_reset"].sum() > 0 and g["out_time_out"].sum() > 0
    np.testing.assert_allclose(ep_means.cpu().numpy(), g["out_extras_episode"], rtol=1e-5, atol=1e-5)
    assert not got["episode_acc"].any()  # zeroed for the next step
    # the oracle on the same inputs: bit-exact
    lib = bridge.ensure_built()
    bridge.set_ground(lib)
    bridge.set_self_collision(lib)
    Eh = bridge._env_struct(host)
    mh = cabi.ModelHandle(spec.model)
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_post_physics(C.byref(mh.desc), C.byref(spec.task), N, p(host["root"]), p(host["dofs"]),
                         p(host["cforce"]), p(host["rbs"]), C.byref(Eh), step)
    assert_exact(got, host, STATE + POST, N, f"{task} golden post-physics vs oracle")
    sim.close()


# ------------------------------------------------------------- fused step --
def warm(task, n, steps=30, seed=0, **edits):
    env = make(task, n, **edits)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(seed)
    for _ in range(steps):
        env.step(0.5 * torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g))
    return env, g


@pytest.mark.parametrize("task", TASKS)
def test_post_physics_on_hip_physics_state_matches_oracle_exactly(task):
    """Decoupled check (no physics tolerance can hide an obs/reward error): the HIP physics
    half runs, then the HIP post half and the ORACLE post half both run on the HIP's own
    post-substep state.  Every env, every output: exact."""
    env, g = warm(task, 512)
    for it in range(3):
        a = 0.5 * torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g)
        env._sync_stream()
        env._buf_idx ^= 1
        E = env._env_structs[env._buf_idx]
        env.actions.copy_(a)
        E.actions_in = None
        E.ep_snapshot = None
        step = env.common_step_counter
        env.sim.step_physics(E, step)
        snap = bridge.snapshot(env)  # the HIP physics half's state + the post half's inputs
        env.sim.post_physics(E, step)
        env._step_mirror += 1
        env.obs_buf, env.privileged_obs_buf = env._obs_bufs[env._buf_idx], env._priv_bufs[env._buf_idx]
        env.reset_buf, env.time_out_buf = env._reset_bufs[env._buf_idx], env._timeout_bufs[env._buf_idx]
        got = env_arrays(env)
        ref = bridge_post(env, snap, step)
        assert_exact(got, ref, STATE + POST, env.num_envs, f"{task} post-physics step {it}")


def bridge_post(env, snap, step):
    lib = bridge.ensure_built()
    bridge.set_env(lib, env)
    b = {k: (None if v is None else np.ascontiguousarray(v).copy()) for k, v in snap.items()}
    b["episode_acc"][:] = 0
    mh = cabi.ModelHandle(env.model)
    E = bridge._env_struct(b)
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_post_physics(C.byref(mh.desc), C.byref(env.task_params), env.num_envs, p(b["root"]), p(b["dofs"]),
                         p(b["cforce"]), p(b["rbs"]) if writes_body_states(env) else None, C.byref(E), int(step))
    return b


ENV_TENSORS = ["root_states", "dof_state", "_contact_forces", "rigid_body_states", "actions", "last_actions",
               "last_dof_vel", "last_root_vel", "torques", "commands", "feet_air_time", "last_contacts",
               "_episode_length", "rew_buf", "_episode_sums", "_episode_acc", "base_lin_vel", "base_ang_vel",
               "projected_gravity", "rpy", "phase", "leg_phase", "_d_step_counter", "_ep_means", "_time_outs"]


def save(env):
    out = {k: getattr(env, k).clone() for k in ENV_TENSORS}
    for name in ("_obs_bufs", "_priv_bufs", "_reset_bufs", "_timeout_bufs"):
        out[name] = [None if t is None else t.clone() for t in getattr(env, name)]
    out["_buf_idx"], out["_step_mirror"] = env._buf_idx, env._step_mirror
    return out


def restore(env, st):
    for k in ENV_TENSORS:
        getattr(env, k).copy_(st[k])
    for name in ("_obs_bufs", "_priv_bufs", "_reset_bufs", "_timeout_bufs"):
        for t, s in zip(getattr(env, name), st[name]):
            if t is not None:
                t.copy_(s)
    env._buf_idx, env._step_mirror = st["_buf_idx"], st["_step_mirror"]


@pytest.mark.parametrize("task", TASKS)
def test_fused_step_is_physics_then_post_bitwise(task):
    env, g = warm(task, 256)
    a = 0.5 * torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g)
    st = save(env)
    env.step(a)
    fused = env_arrays(env)
    restore(env, st)
    env._buf_idx ^= 1
    E = env._env_structs[env._buf_idx]
    env.actions.copy_(a)
    E.actions_in = None
    E.ep_snapshot = None
    env.sim.step_physics(E, env.common_step_counter)
    env.sim.post_physics(E, env.common_step_counter)
    env._step_mirror += 1
    env.obs_buf, env.privileged_obs_buf = env._obs_bufs[env._buf_idx], env._priv_bufs[env._buf_idx]
    env.reset_buf, env.time_out_buf = env._reset_bufs[env._buf_idx], env._timeout_bufs[env._buf_idx]
    split = env_arrays(env)
    assert_exact(split, fused, STATE + POST, env.num_envs, f"{task} fused vs split")
    assert int(env._d_step_counter) == st["_step_mirror"] + 1


def fused_vs_oracle(env, g, steps, what):
    for it in range(steps):
        snap = bridge.snapshot(env)
        a = 0.5 * torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g)
        ref = bridge.step(env, snap, a.cpu().numpy(), env.common_step_counter)
        env.step(a)
        got = env_arrays(env)
        assert_exact(got, ref, STATE + POST, env.num_envs, f"{what} step {it}",
                     skip_body_states=not writes_body_states(env))


@pytest.mark.parametrize("task", TASKS)
def test_fused_step_matches_oracle_bitwise(task):
    env, g = warm(task, 512)
    # the chain-structured instantiations eliminate the chains' joint pivots level by level;
    # bridge.step hands that order to the oracle (orc_set_factor_chain)
    assert env.sim.factor_chain() == {"go2": 3, "h1": 5, "g1": 6, "h1_2": 6}[task]
    fused_vs_oracle(env, g, 3, task)


@pytest.mark.parametrize("task,n", [("go2", 1), ("go2", 4), ("go2", 6), ("h1", 2), ("go2", 37), ("h1_2", 65),
                                    ("go2", 4096), ("h1", 8192), ("g1", 4096), ("h1_2", 8192)])
def test_fused_step_matches_oracle_bitwise_edge_and_full_sizes(task, n):
    """Ragged env counts (partial XCD-mapped waves) and the BASELINE per-GPU sizes.  Go2 at 4
    envs is BASELINE configs[0]'s size; 4, 6 and 2 envs run two envs per wave on fewer
    workgroups than the 8 XCDs xcd_env() deals over.  h1_2 at 65 envs, seed 65, is the case
    whose one-env torque mismatch round 1 hid behind a 1/n allowance (fp contraction + libm vs
    ocml last-bit differences); it is exact now."""
    env, g = warm(task, n, steps=8, seed=n)
    fused_vs_oracle(env, g, 2, f"{task} x{n}")


@pytest.mark.parametrize("task", ["go2", "g1_rough"])
def test_heightfield_step_matches_oracle_bitwise(task):
    env, g = warm(task, 512, terrain__mesh_type="heightfield", terrain__num_rows=5, terrain__num_cols=8)
    fused_vs_oracle(env, g, 3, task)
    bridge.set_ground(bridge.ensure_built())


def test_g1_rough_at_its_baseline_size_matches_oracle_bitwise():
    """BASELINE configs[2] as benched: G1, 4096 envs, the default curriculum map (10 x 20
    tiles of 8 m at 0.1 m + 25 m border: int16 1300 x 2100, legged_robot_config.py:63-87),
    envs spread over every tile row (rows = difficulty levels)."""
    env, g = warm("g1_rough", 4096, steps=8, seed=4096)
    assert env.height_samples.shape == (1300, 2100)
    fused_vs_oracle(env, g, 2, "g1_rough x4096 default map")
    bridge.set_ground(bridge.ensure_built())


@pytest.mark.parametrize("task", ["go2", "h1"])
def test_reset_idx_subset_matches_oracle(task):
    """reset_idx(env_ids) for a random subset (legged_robot.py:723-768): the masked launch
    == the oracle's reset of the same envs; the other envs are untouched; extras["episode"]
    = mean of the reset envs' episode sums / episode_length_s; reset_buf[env_ids] = 1."""
    env, g = warm(task, 256, steps=40)
    ids = torch.randperm(env.num_envs, generator=torch.Generator().manual_seed(3))[:57].cuda()
    snap = bridge.snapshot(env)
    i = env._buf_idx  # reset_idx writes the CURRENT buffers
    snap["reset"] = env._reset_bufs[i].cpu().numpy().astype(np.uint8)
    before = env_arrays(env)
    sums_before = env._episode_sums.cpu().numpy().copy()
    env.reset_idx(ids)
    got = env_arrays(env)
    lib = bridge.ensure_built()
    b = {k: (None if v is None else np.ascontiguousarray(v).copy()) for k, v in snap.items()}
    b["episode_acc"][:] = 0
    mask = np.zeros(env.num_envs, np.uint8)
    mask[ids.cpu().numpy()] = 1
    E = bridge._env_struct(b)
    mh = cabi.ModelHandle(env.model)
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_reset_idx(C.byref(mh.desc), C.byref(env.task_params), env.num_envs, p(b["root"]), p(b["dofs"]),
                      C.byref(E), p(mask), int(env.common_step_counter))
    keys = ["root", "dofs", "commands", "actions", "last_actions", "last_dof_vel", "feet_air_time",
            "episode_length", "episode_sums", "reset"]
    assert_exact(got, b, keys, env.num_envs, f"{task} reset_idx")
    keep = mask == 0
    for k in ("root", "dofs", "commands", "episode_length", "obs"):
        np.testing.assert_array_equal(per_env(got[k], env.num_envs)[keep], per_env(before[k], env.num_envs)[keep])
    assert (got["reset"][mask == 1] == 1).all()
    ep = env.extras["episode"]
    want = sums_before[:, mask == 1].mean(axis=1) / env.max_episode_length_s
    have = np.array([float(ep["rew_" + k]) for k in env._sum_names])
    np.testing.assert_allclose(have, want, rtol=1e-5, atol=1e-7)


def test_two_envs_per_wave_is_bitwise_one_env_per_wave(monkeypatch):
    """k_step carries two Go2 envs per wave (lanes 0-31 / 32-63) at even env counts; the
    one-env-per-wave kernel (LGS_ENVS_PER_WAVE=1, read at lgs_create_sim) must give the same
    bits for every buffer over a rollout with resets."""
    outs = []
    for epw in ("1", "2"):
        monkeypatch.setenv("LGS_ENVS_PER_WAVE", epw)
        env, g = warm("go2", 512, steps=60, seed=11)
        outs.append(env_arrays(env))
        env.close()
    assert_exact(outs[1], outs[0], STATE + POST, 512, "two envs per wave vs one")


@pytest.mark.parametrize("task", ["h1", "g1", "h1_2"])
def test_humanoid_two_envs_per_wave_is_bitwise_one_env_per_wave(task, monkeypatch):
    """The humanoids' 32-row capacity (8 contact slots, 8 limit rows) runs two envs per wave
    like Go2; it must equal the oracle bit for bit and the one-env-per-wave build of the same
    capacity over a rollout with resets."""
    outs = []
    for epw in ("1", "2"):
        monkeypatch.setenv("LGS_ENVS_PER_WAVE", epw)
        env, g = warm(task, 256, steps=40, seed=5)
        outs.append(env_arrays(env))
        if epw == "2":
            fused_vs_oracle(env, g, 2, f"{task} 32 rows")
        env.close()
    assert_exact(outs[1], outs[0], STATE + POST, 256, f"{task} 32 rows: two envs per wave vs one")


# --------------------------------------------------- another robot (plugin) --
def _register_g1_23dof():
    """A plugin task on a robot the built-in kernels do not cover: the G1 23-DOF description
    the reference ships (resources/robots/g1_description/g1_23dof.urdf; the bundled model
    leggedsim/models/g1_23dof.npz is compiled from it).  Its (23 DOFs, 24 bodies) shape comes
    from the library's build-time instantiation hook (LGS_EXTRA_SHAPES in csrc/leggedsim.hip)."""
    import copy
    from legged_gym.envs.g1.g1_config import G1RoughCfg, G1RoughCfgPPO
    from legged_gym.envs.g1.g1_env import G1Robot
    if "g1_23dof" in task_registry.task_classes:
        return
    cfg = copy.deepcopy(G1RoughCfg())
    cfg.asset.file = "{LEGGED_GYM_ROOT_DIR}/resources/robots/g1_description/g1_23dof.urdf"
    cfg.asset.self_collisions = 1
    arms = {"waist_yaw_joint": 0.0}
    for side in ("left", "right"):
        arms.update({f"{side}_shoulder_pitch_joint": 0.3, f"{side}_shoulder_roll_joint": 0.25 * (1 if side == "left" else -1),
                     f"{side}_shoulder_yaw_joint": 0.0, f"{side}_elbow_joint": 0.9, f"{side}_wrist_roll_joint": 0.0})
    cfg.init_state.default_joint_angles = dict(cfg.init_state.default_joint_angles, **arms)
    cfg.control.stiffness = dict(cfg.control.stiffness, waist=150, shoulder=40, elbow=40, wrist=20)
    cfg.control.damping = dict(cfg.control.damping, waist=3, shoulder=1, elbow=1, wrist=0.5)
    cfg.env.num_actions = 23
    cfg.env.num_observations = 9 + 3 * 23 + 2
    cfg.env.num_privileged_obs = 12 + 3 * 23 + 2
    task_registry.register("g1_23dof", G1Robot, cfg, G1RoughCfgPPO())


@pytest.mark.parametrize("n", [37, 1024])
def test_other_robot_shape_registers_and_matches_oracle_bitwise(n):
    """configs' robots aside: a task on another robot (23 DOFs, 24 bodies, humanoid
    observations of 80 / 83 entries) registers, steps through the same C ABI and is
    bit-exact with the oracle; name queries resolve its bodies."""
    _register_g1_23dof()
    env, g = warm("g1_23dof", n, steps=6, seed=n)
    assert env.num_dof == 23 and env.num_bodies == 24 and env.obs_buf.shape == (n, 80)
    assert env.sim.find_body("torso_link") == env.model.body_names.index("torso_link")
    fused_vs_oracle(env, g, 2, f"g1_23dof x{n}")


@pytest.mark.parametrize("task", ["h1", "g1"])
def test_step_refreshes_the_feet_rows_and_gym_refresh_every_body(task):
    """The humanoid step refreshes the rigid_body_states rows its task reads (the feet,
    h1_env.py:34-52: lgs_task_params.body_state_mask); the other rows stay as they were.
    gym.refresh_rigid_body_state_tensor (lgs_forward_kinematics) then refreshes every row,
    equal to the oracle's forward kinematics of the same state."""
    import ctypes as C
    env, g = warm(task, 64, steps=5)
    B = env.num_bodies
    feet = env.feet_indices.cpu().numpy()
    other = np.setdiff1d(np.arange(B), feet)
    env.rigid_body_states.fill_(7.0)
    env.step(0.5 * torch.randn(env.num_envs, env.num_actions, device="cuda", generator=g))
    rbs = env.rigid_body_states.view(env.num_envs, B, 13).cpu().numpy()
    assert (rbs[:, other] == 7.0).all() and not (rbs[:, feet] == 7.0).any()
    feet_rows = rbs[:, feet].copy()
    env.gym.refresh_rigid_body_state_tensor(env.sim)
    rbs = env.rigid_body_states.view(env.num_envs, B, 13).cpu().numpy()
    np.testing.assert_array_equal(rbs[:, feet], feet_rows)
    lib = bridge.ensure_built()
    mh = cabi.ModelHandle(env.model)
    root = env.root_states.cpu().numpy()
    dofs = env.dof_state.cpu().numpy().reshape(env.num_envs, -1)
    want = np.zeros((env.num_envs, B, 13), np.float32)
    for e in range(env.num_envs):
        r, d = np.ascontiguousarray(root[e]), np.ascontiguousarray(dofs[e])
        lib.orc_body_states_env(C.byref(mh.desc), r.ctypes.data, d.ctypes.data, want[e].ctypes.data)
    np.testing.assert_array_equal(rbs, want)
