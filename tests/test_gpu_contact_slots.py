"""Non-foot bodies on the ground, through the fused HIP step, bit-exact with the oracle.

Humanoids kneeling and sitting (tests/golden/contact_poses.npz, tools/make_contact_poses.py):
both feet plus a knee, then plus the pelvis, on the ground.  The reference reads those bodies'
contact forces: check_termination the pelvis (legged_robot.py:711-721, h1_config.py:76),
_reward_collision the hips and knees (legged_robot.py:877-879, h1_config.py:75).  The slot
policy (include/leggedsim.h, above lgs_self_collision_desc) gives every touching body a
contact row before further sole corners, so:

* a knee on the ground carries a normal force while both feet are planted,
* H1's `collision` term fires on it,
* the pelvis on the ground resets the env,
* HIP == oracle for every buffer, every env, and the capacity counters
  (lgs_get_contact_stats) equal the oracle's.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import bridge  # noqa: E402
from conftest import GOLDEN  # noqa: E402
from leggedsim import cabi  # noqa: E402
from test_gpu_parity import POST, STATE, assert_exact, env_arrays, make, writes_body_states  # noqa: E402

POSES = [(r, p) for r in ("h1", "g1", "h1_2") for p in ("kneel", "sit")]


def place(env, task, pose, vz=-0.2, q=None, qd=None):
    """Every env in the pose (at its own origin), pressing into the ground at vz; returns the
    actions whose PD targets are the pose."""
    z = np.load(f"{GOLDEN}/contact_poses.npz")
    dev = env.device
    root = torch.tensor(z[f"{task}_{pose}_root"], device=dev)
    qp = torch.tensor(z[f"{task}_{pose}_q"] if q is None else q, device=dev, dtype=torch.float)
    env.root_states[:] = root
    env.root_states[:, :2] += env.env_origins[:, :2]
    env.root_states[:, 9] = vz
    env.dof_pos[:] = qp
    env.dof_vel[:] = 0.0 if qd is None else torch.as_tensor(qd, device=dev, dtype=torch.float)
    a = (qp - env.default_dof_pos.view(-1)) / env.cfg.control.action_scale
    return a.expand(env.num_envs, env.num_actions).contiguous()


def step_vs_oracle(env, a):
    """One fused step on the GPU and on the oracle from the same state: every buffer, the
    per-term rewards and the capacity counters equal."""
    N = env.num_envs
    lib = bridge.ensure_built()
    cnt = np.zeros(cabi.NUM_CONTACT_STATS, np.uint64)
    lib.orc_contact_stats(cnt.ctypes.data, 1)
    env.sim.contact_stats(reset=True)
    nr = len(env._native_reward_names)
    rt = torch.zeros(nr, N, device=env.device)
    for E in env._env_structs:
        E.rew_terms = rt.data_ptr()
    snap = bridge.snapshot(env)
    snap["rew_terms"] = np.zeros((nr, N), np.float32)
    ref = bridge.step(env, snap, a.cpu().numpy(), env.common_step_counter)
    env.step(a)
    got = env_arrays(env)
    for E in env._env_structs:
        E.rew_terms = None
    got["rew_terms"] = rt.cpu().numpy()
    assert_exact(got, ref, STATE + POST + ["rew_terms"], N, "contact pose", skip_body_states=not writes_body_states(env))
    lib.orc_contact_stats(cnt.ctypes.data, 1)
    hip = env.sim.contact_stats(reset=True)
    assert [hip["bodies"], hip["self"], hip["limits"]] == [int(x) for x in cnt]
    return got, hip


@pytest.mark.parametrize("task,pose", POSES)
def test_knee_and_pelvis_contacts_with_planted_feet(task, pose):
    env = make(task, 64)
    env.reset()
    a = place(env, task, pose)
    got, hip = step_vs_oracle(env, a)
    names = env.body_names
    cf = got["cforce"].reshape(env.num_envs, env.num_bodies, 3)
    fn = np.linalg.norm(cf, axis=2)
    feet = [names.index(n) for n in names if env.cfg.asset.foot_name in n]
    knees = [i for i, n in enumerate(names) if "knee" in n]
    touching = [int(b) for b in np.load(f"{GOLDEN}/contact_poses.npz")[f"{task}_{pose}_touching"]]
    # the knee(s) of the pose carry load in every env, next to the feet
    assert (fn[:, [k for k in knees if k in touching]].max(axis=1) > 0.0).all()
    if pose == "kneel":  # (sitting, the pelvis and thighs carry the load; a sole may only graze)
        assert (fn[:, feet].max(axis=1) > 0.0).all()
    if pose == "sit":  # the pelvis on the ground: check_termination (> 1 N on a termination body)
        assert (fn[:, 0] > 1.0).all()
        assert got["reset"].all()
    else:
        assert (fn[:, 0] == 0.0).all()
    if task == "h1":  # H1 penalises hip/knee contacts (h1_config.py:75): collision = -1 * count * dt
        k = env._native_reward_names.index("collision")
        assert (got["rew_terms"][k] < 0.0).all()
    if task == "g1" and pose == "sit":  # 10 touching bodies, 8 slots: the two left over are counted
        assert hip["bodies"] > 0
    else:
        assert hip["bodies"] == 0
    env.close()


@pytest.mark.parametrize("task", ["h1", "g1"])
def test_joint_limits_beyond_the_limit_block(task):
    """Every joint past a limit and moving out: in the air the limits beyond the 8-row limit
    block take the rows of the unused contact slots (nothing dropped); sitting, with every
    contact slot taken, the rest is counted; both bit-exact with the oracle."""
    env = make(task, 64)
    env.reset()
    D = env.num_dof
    lo, hi = env.dof_pos_limits[:, 0].cpu().numpy(), env.dof_pos_limits[:, 1].cpu().numpy()
    m = env.model
    q = np.where(np.arange(D) % 2 == 0, m.dof_upper + 0.05, m.dof_lower - 0.05).astype(np.float32)
    qd = np.where(np.arange(D) % 2 == 0, 1.0, -1.0).astype(np.float32)
    assert (q > hi).sum() + (q < lo).sum() == D
    a = place(env, task, "sit", vz=0.0, q=q, qd=qd)
    env.root_states[:, 2] += 3.0  # in the air
    _, hip = step_vs_oracle(env, a)
    assert hip["limits"] == 0
    env.reset()
    a = place(env, task, "sit", q=q, qd=qd)
    _, hip = step_vs_oracle(env, a)
    assert hip["limits"] > 0
    env.close()
