"""The contact-slot policy of the oracle (include/leggedsim.h, above lgs_self_collision_desc),
on humanoid poses with non-foot bodies on the ground (tests/golden/contact_poses.npz, made
by tools/make_contact_poses.py): one slot per touching body first, then self contacts, then
the other touching ground candidates; what does not fit is counted.

PhysX reports a force for every touching shape (check_termination reads the pelvis,
legged_robot.py:715; _reward_collision the hips and knees, :877-879).  The poses are the
cases where filling the slots in candidate order (feet first) left a touching knee or the
pelvis without a row; here every touching body gets one."""
import ctypes as C

import numpy as np
import pytest

import bridge
from conftest import GOLDEN
from hostspec import make_spec
from leggedsim import cabi

POSES = [(r, p) for r in ("h1", "g1", "h1_2") for p in ("kneel", "sit")]


def pose_state(spec, task, pose, vz=-0.2):
    z = np.load(f"{GOLDEN}/contact_poses.npz")
    root = z[f"{task}_{pose}_root"].reshape(1, 13).copy()
    root[0, 9] = vz  # pressing into the ground: every touching candidate's row engages
    dofs = np.zeros((spec.num_dof, 2), np.float32)
    dofs[:, 0] = z[f"{task}_{pose}_q"]
    return root, dofs, [int(b) for b in z[f"{task}_{pose}_touching"]]


def candidates(lib, spec, root, dofs):
    """World candidate points (sphere centres) and their separation from the plane, in the
    env's candidate order (feet first, Model.reorder_points)."""
    mh = cabi.ModelHandle(spec.model)
    m = spec.model
    rbs = np.zeros((m.num_bodies, 13), np.float32)
    lib.orc_body_states_env(C.byref(mh.desc), root.ctypes.data, dofs.ctypes.data, rbs.ctypes.data)
    pts = np.zeros((m.num_points, 3))
    for k, b in enumerate(m.pt_body):
        x, y, zq, w = rbs[b, 3:7].astype(np.float64)
        R = np.array([[1 - 2 * (y * y + zq * zq), 2 * (x * y - zq * w), 2 * (x * zq + y * w)],
                      [2 * (x * y + zq * w), 1 - 2 * (x * x + zq * zq), 2 * (y * zq - x * w)],
                      [2 * (x * zq - y * w), 2 * (y * zq + x * w), 1 - 2 * (x * x + y * y)]])
        pts[k] = rbs[b, :3] + R @ m.pt_pos[k]
    sep = pts[:, 2] - m.pt_radius - spec.sim_params.rest_offset
    return pts, sep


def slot_bodies(spec, sep):
    """The slot policy restated: primaries (first touching candidate per body), then the rest."""
    m, maxc = spec.model, spec.sim_params.max_contacts
    act = np.nonzero(sep < spec.sim_params.contact_offset)[0]
    seen, prim, rest = set(), [], []
    for k in act:
        b = int(m.pt_body[k])
        (rest if b in seen else prim).append(k)
        seen.add(b)
    slots = (prim[:maxc] + rest)[:maxc]
    return act, prim, slots


@pytest.mark.parametrize("task,pose", POSES)
def test_every_touching_body_gets_a_contact_row(task, pose, oracle_lib):
    spec = make_spec(task)
    root, dofs, touching = pose_state(spec, task, pose)
    pts, sep = candidates(oracle_lib, spec, root, dofs)
    act, prim, slots = slot_bodies(spec, sep)
    m = spec.model
    bodies = sorted({int(m.pt_body[k]) for k in act})
    assert set(touching) <= set(bodies)  # (the generator listed the bodies within 5 mm)
    knees = [b for b in bodies if "knee" in m.body_names[b]]
    assert knees, "every pose puts a knee on the ground"
    if pose == "sit" and task != "h1_2":
        # the case the policy exists for: the first max_contacts touching candidates in
        # candidate order (feet, then the pelvis's many hull points; H1_2's pelvis is a box
        # of 8 corners) leave a knee out
        first = {int(m.pt_body[k]) for k in act[: spec.sim_params.max_contacts]}
        assert not set(knees) <= first
    bridge.set_self_collision(oracle_lib, None)
    oracle_lib.orc_set_heightfield(None, 0, 0, 0.0, 0.0, 0.0)
    stats = np.zeros(cabi.NUM_CONTACT_STATS, np.uint64)
    oracle_lib.orc_contact_stats(stats.ctypes.data, 1)
    mh = cabi.ModelHandle(spec.model)
    B = spec.num_bodies
    cf = np.zeros((B, 3), np.float32)
    rbs = np.zeros((B, 13), np.float32)
    tau = np.zeros((1, spec.num_dof), np.float32)
    p = lambda a: a.ctypes.data  # noqa: E731
    oracle_lib.orc_simulate(C.byref(mh.desc), C.byref(spec.sim_params), 1, p(root), p(dofs), p(tau), p(cf), p(rbs),
                            None, None)
    oracle_lib.orc_contact_stats(stats.ctypes.data, 1)
    maxc = spec.sim_params.max_contacts
    assert int(stats[0]) == max(0, len(bodies) - maxc)  # bodies left without a slot
    slotted = {int(m.pt_body[k]) for k in slots}
    assert len(slotted) == min(len(bodies), maxc)
    for b in set(bodies) - slotted:  # no row, no force (what the counter reports)
        assert not cf[b].any()
    # pressed into the ground at 0.2 m/s the slotted knee(s) push back (a slotted contact may
    # legitimately end with zero force when others carry the load, so only the knees are asserted)
    assert any(cf[b, 2] > 0.0 for b in knees if b in slotted)
    assert cf[:, 2].sum() > 0.0


@pytest.mark.parametrize("task", ["h1", "g1"])
def test_limits_beyond_the_limit_block_use_free_contact_rows(task, oracle_lib):
    """Every joint past its limit in the air: D > 8 limit rows, so the limits after the first
    8 take the rows of the (unused) contact slots and none is dropped; on the ground with all
    slots taken the rest is counted."""
    spec = make_spec(task)
    D = spec.num_dof
    m = spec.model
    bridge.set_self_collision(oracle_lib, None)
    oracle_lib.orc_set_heightfield(None, 0, 0, 0.0, 0.0, 0.0)
    mh = cabi.ModelHandle(m)
    p = lambda a: a.ctypes.data  # noqa: E731
    stats = np.zeros(cabi.NUM_CONTACT_STATS, np.uint64)
    for z0, want_drop in ((5.0, False), (None, True)):
        if z0 is None:  # the sit pose: every slot taken by ground contacts
            root, dofs, _ = pose_state(spec, task, "sit")
            _, sep = candidates(oracle_lib, spec, root, dofs)
            assert (sep < spec.sim_params.contact_offset).sum() >= spec.sim_params.max_contacts
        else:
            root = np.zeros((1, 13), np.float32)
            root[0, 2], root[0, 6] = z0, 1.0
            dofs = np.zeros((D, 2), np.float32)
        # every joint 0.05 rad past a limit, moving further out
        dofs[:, 0] = np.where(np.arange(D) % 2 == 0, m.dof_upper + 0.05, m.dof_lower - 0.05)
        dofs[:, 1] = np.where(np.arange(D) % 2 == 0, 1.0, -1.0)
        q0 = dofs[:, 0].copy()
        oracle_lib.orc_contact_stats(stats.ctypes.data, 1)
        cf = np.zeros((spec.num_bodies, 3), np.float32)
        rbs = np.zeros((spec.num_bodies, 13), np.float32)
        tau = np.zeros((1, D), np.float32)
        oracle_lib.orc_simulate(C.byref(mh.desc), C.byref(spec.sim_params), 1, p(root), p(dofs), p(tau), p(cf),
                                p(rbs), None, None)
        oracle_lib.orc_contact_stats(stats.ctypes.data, 1)
        lim_rows = spec.sim_params.max_rows - 3 * spec.sim_params.max_contacts
        if want_drop:
            assert int(stats[2]) == D - lim_rows
        else:
            assert int(stats[2]) == 0
            # every limit row pushed its joint back inside: velocity turned towards the range
            assert (np.sign(dofs[:, 1]) != np.sign(np.where(np.arange(D) % 2 == 0, 1.0, -1.0))).all() or \
                (np.abs(dofs[:, 0] - q0) < 0.05).all()
