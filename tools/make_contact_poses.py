"""Generate tests/golden/contact_poses.npz: humanoid states with non-foot bodies on the ground.

For H1, G1 and H1_2 (the bundled models, leggedsim/models/*.npz) two poses are searched
(joint angles inside the URDF limits, root height/pitch free):

* ``kneel``: the left sole flat on the ground, the right knee and the right foot down
  (a one-knee kneel; G1, whose legs cannot reach it: both knees and both feet), pelvis in
  the air;
* ``sit``: the pelvis, both knees (backs of the legs) and both heels on the ground.

The search is a derivative-free minimisation over the lowest candidate point of each
target body (forward kinematics in numpy, the model's own conventions).  Each pose is
shifted so its deepest candidate sits 2 mm below the ground (inside contact_offset).
Stored per robot and pose: root_states[13] (xyzw quaternion, zero velocity), dof q[D],
and which bodies touch.  These are inputs for tests/test_gpu_contact_slots.py, not
reference outputs.

    python tools/make_contact_poses.py
"""
import os
import sys

import numpy as np
from scipy.optimize import minimize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
from leggedsim.model import Model  # noqa: E402

ROBOTS = {"h1": "h1", "g1": "g1_12dof", "h1_2": "h1_2_12dof"}
FOOT = {"h1": "ankle", "g1": "ankle_roll", "h1_2": "ankle_roll"}


def axis_angle(a, t):
    a = np.asarray(a, np.float64)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


def fk(m, pos, pitch, q):
    """World candidate points (bottom of each sphere) and their bodies."""
    B = m.num_bodies
    R = [None] * B
    p = [None] * B
    R[0] = axis_angle([0, 1, 0], pitch)
    p[0] = np.asarray(pos, np.float64)
    for b in range(1, B):
        P = m.parent[b]
        Rj = R[P] @ m.joint_rot[b].reshape(3, 3).astype(np.float64)
        p[b] = p[P] + R[P] @ m.joint_pos[b]
        j = m.dof[b]
        R[b] = Rj @ axis_angle(m.axis[b], q[j]) if j >= 0 else Rj
    pts = np.empty((m.num_points, 3))
    for b in range(B):
        sel = _sel(m, b)
        pts[sel] = p[b] + m.pt_pos[sel].astype(np.float64) @ R[b].T
    pts[:, 2] -= m.pt_radius
    return pts


def _sel(m, b):
    if not hasattr(m, "_pts_of"):
        m._pts_of = [np.nonzero(m.pt_body == x)[0] for x in range(m.num_bodies)]
    return m._pts_of[b]


def body_min(m, pts, b):
    sel = m.pt_body == b
    return pts[sel, 2].min() if sel.any() else np.inf


def search(m, name, pose, seed):
    D = m.num_dofs
    names = m.dof_names
    idx = {n: i for i, n in enumerate(names)}
    lo, hi = m.dof_lower.astype(np.float64), m.dof_upper.astype(np.float64)
    bid = {n: i for i, n in enumerate(m.body_names)}
    feet = [b for b, n in enumerate(m.body_names) if FOOT[name] in n]
    lfoot = [b for b in feet if "left" in m.body_names[b]][0]
    rfoot = [b for b in feet if "right" in m.body_names[b]][0]
    lknee, rknee = bid["left_knee_link"], bid["right_knee_link"]
    pelvis = 0
    free = [idx[f"{s}_hip_pitch_joint"] for s in ("left", "right")] + \
           [idx[f"{s}_knee_joint"] for s in ("left", "right")] + \
           [idx[n] for n in names if "ankle" in n and ("pitch" in n or n.endswith("ankle_joint"))] + \
           [idx[f"{s}_hip_roll_joint"] for s in ("left", "right")]
    if pose == "kneel" and name == "g1":  # G1's legs cannot reach a one-knee kneel: both knees
        targets, lifted = [lfoot, rfoot, lknee, rknee], [pelvis]
    elif pose == "kneel":
        targets, lifted = [lfoot, rknee, rfoot], [pelvis, lknee]
    else:
        targets, lifted = [pelvis, lknee, rknee, lfoot, rfoot], []

    def unpack(x):
        q = np.zeros(D)
        q[free] = np.clip(x[2:], lo[free], hi[free])
        return x[0], x[1], q

    def cost(x):
        z, pitch, q = unpack(x)
        pts = fk(m, [0, 0, z], pitch, q)
        c = sum(body_min(m, pts, b) ** 2 for b in targets)
        c += sum(max(0.0, 0.08 - body_min(m, pts, b)) ** 2 for b in lifted)
        c += max(0.0, -pts[:, 2].min()) ** 2 * 10
        if pose == "kneel" and name != "g1":  # left sole flat: its lowest candidates level
            sel = m.pt_body == lfoot
            zz = np.sort(pts[sel, 2])[:4]
            c += 0.25 * (zz[-1] - zz[0]) ** 2
        return c

    rng = np.random.default_rng(seed)
    best = None
    for trial in range(80):
        if best is not None and best.fun < 1e-6:
            break
        x0 = np.concatenate([[rng.uniform(0.2, 0.9), rng.uniform(-0.3, 0.3)],
                             rng.uniform(lo[free], hi[free])])
        if pose == "kneel" and trial % 2 == 0:  # a kneeling seed: left leg forward, right shin back
            q0 = np.zeros(D)
            q0[idx["left_hip_pitch_joint"]] = -1.4 if name != "g1" else 0.0
            q0[idx["left_knee_joint"]] = 1.4 if name != "g1" else 1.6
            q0[idx["right_hip_pitch_joint"]] = 0.0
            q0[idx["right_knee_joint"]] = 1.6
            x0 = np.concatenate([[0.4 + 0.01 * (trial % 40), 0.0], np.clip(q0[free] + rng.normal(0, 0.2, len(free)),
                                                                   lo[free], hi[free])])
        if pose == "sit" and trial % 2 == 0:  # a sitting seed: hips flexed, legs straight forward
            q0 = np.zeros(D)
            for s in ("left", "right"):
                q0[idx[f"{s}_hip_pitch_joint"]] = -1.5
            x0 = np.concatenate([[0.15, 0.0], np.clip(q0[free] + rng.normal(0, 0.2, len(free)), lo[free], hi[free])])
        r = minimize(cost, x0, method="Powell", options={"maxiter": 4000, "xtol": 1e-7, "ftol": 1e-12})
        if best is None or r.fun < best.fun:
            best = r
    z, pitch, q = unpack(best.x)
    pts = fk(m, [0, 0, z], pitch, q)
    z -= pts[:, 2].min() + 0.002  # deepest candidate 2 mm into the ground
    pts = fk(m, [0, 0, z], pitch, q)
    touching = sorted({int(m.pt_body[k]) for k in np.nonzero(pts[:, 2] < 0.005)[0]})
    return z, pitch, q, touching, best.fun


def main():
    out = {}
    for name, stem in ROBOTS.items():
        m = Model.load(os.path.join(ROOT, "unitree-rl-gym_amd", "leggedsim", "models", stem + ".npz"))
        for pose in ("kneel", "sit"):
            z, pitch, q, touching, cost = search(m, name, pose, seed=len(name) + len(pose))
            root = np.zeros(13, np.float32)
            root[2] = z
            root[3:7] = [0.0, np.sin(pitch / 2), 0.0, np.cos(pitch / 2)]  # xyzw, about y
            out[f"{name}_{pose}_root"] = root
            out[f"{name}_{pose}_q"] = q.astype(np.float32)
            out[f"{name}_{pose}_touching"] = np.array(touching, np.int32)
            print(f"{name:5s} {pose:5s} cost {cost:.2e} z {z:.3f} pitch {pitch:+.2f} touching "
                  f"{[m.body_names[b] for b in touching]}")
    path = os.path.join(ROOT, "tests", "golden", "contact_poses.npz")
    np.savez(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
