"""Self-collision between the links of one actor.

IsaacGym's ``create_actor(env, asset, pose, name, i, self_collisions, 0)`` collision
filter (reference ``legged_gym/envs/base/legged_robot.py:373-374``) lets links of one
articulation collide with each other when ``cfg.asset.self_collisions == 0`` -- the
G1/H1/H1_2 configs (``g1_config.py:65``, ``h1_config.py:77``, ``h1_2_config.py:86``) and
``LeggedRobotCfg``; Go2 sets 1 (filtered).  PhysX never tests links joined by a joint.

The model here: every collision shape (URDF ``<collision>`` element; a link merged by
fixed-joint collapse keeps each of its shapes) gets ONE capsule proxy, the tightest
capsule along the principal axis of the shape's contact-candidate points (mesh hull
support points, sphere/capsule centres with their radii, box corners) that encloses them
all.  Candidate pairs are proxies on links that are not the same link and not parent and
child (PhysX's joint filter).  Two pre-filters run once at env creation: pairs whose
proxies already overlap in the default pose are dropped -- a proxy is fatter than the mesh it
encloses, and a pair touching at rest would push the robot apart from the first substep (e.g.
a hip link and the pelvis it is mounted in); and pairs that stay apart over a dense random
sample of the joint box (``reach_samples`` poses uniform within the URDF limits) are dropped
as unreachable -- the static broadphase that keeps the per-substep test to a few dozen pairs
(G1's head never meets its ankles).  The simulator tests the remaining pairs every substep
(``lgs_set_self_collision``): closest points of the two capsule segments, one contact
(normal + friction pair, shape friction) per touching pair.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

MAX_PAIRS = 192    # LGS_MAX_SELF_PAIRS: up to three 64-lane passes in the HIP kernel
MAX_PROXIES = 64   # LGS_MAX_SELF_PROXIES


def capsule_proxies(model):
    """Per collision shape: body index [S] int32 and capsule [S, 7] float32 (p0 xyz, p1 xyz,
    radius) in the body frame."""
    shapes = model.pt_shape if model.pt_shape is not None else model.pt_body
    ids = sorted(set(int(x) for x in shapes))
    caps = np.zeros((len(ids), 7), dtype=np.float64)
    body = np.zeros(len(ids), dtype=np.int32)
    for k, sid in enumerate(ids):
        sel = shapes == sid
        body[k] = int(model.pt_body[sel][0])
        P = model.pt_pos[sel].astype(np.float64)
        rad = model.pt_radius[sel].astype(np.float64)
        c = P.mean(axis=0)
        if len(P) > 1 and np.ptp(P, axis=0).max() > 0:
            w, V = np.linalg.eigh(np.cov((P - c).T))
            ax = V[:, -1]
        else:
            ax = np.array([0.0, 0.0, 1.0])
        t = (P - c) @ ax
        perp = np.linalg.norm((P - c) - np.outer(t, ax), axis=1)
        r = float((perp + rad).max())
        # tightest segment for this axis and radius: point k is inside the capsule when its
        # projection lies on the segment or it is within r of the nearer end
        slack = np.sqrt(np.maximum(r * r - (perp + rad) ** 2, 0.0))
        t0, t1 = float((t + slack).min()), float((t - slack).max())
        if t0 > t1:
            t0 = t1 = 0.5 * (t0 + t1)
        # the radius that encloses every point around the chosen segment (exact for t0 <= t1
        # by construction; grows when the segment collapsed to its midpoint)
        tt = np.clip(t, t0, t1)
        r = max(r, float((np.linalg.norm((P - c) - np.outer(tt, ax), axis=1) + rad).max()))
        caps[k, 0:3] = c + t0 * ax
        caps[k, 3:6] = c + t1 * ax
        caps[k, 6] = r
    return body, caps.astype(np.float32)


def _axis_angle(a, ang):
    s, c = math.sin(ang), math.cos(ang)
    t = 1.0 - c
    x, y, z = a
    return np.array([[t * x * x + c, t * x * y - s * z, t * x * z + s * y],
                     [t * x * y + s * z, t * y * y + c, t * y * z - s * x],
                     [t * x * z - s * y, t * y * z + s * x, t * z * z + c]])


def body_frames(model, q):
    """World rotation [B,3,3] and origin [B,3] of every body for joint angles q, root at
    the origin with identity orientation (the simulator's forward kinematics)."""
    B = model.num_bodies
    R = np.zeros((B, 3, 3))
    p = np.zeros((B, 3))
    R[0] = np.eye(3)
    for b in range(1, B):
        a = model.parent[b]
        Rj = R[a] @ model.joint_rot[b].reshape(3, 3).astype(np.float64)
        p[b] = p[a] + R[a] @ model.joint_pos[b].astype(np.float64)
        j = model.dof[b]
        R[b] = Rj @ _axis_angle(model.axis[b].astype(np.float64), float(q[j])) if j >= 0 else Rj
    return R, p


def segment_closest(p1, q1, p2, q2):
    """Closest points of segments p1q1 and p2q2 (Ericson, Real-Time Collision Detection 5.1.9)."""
    d1, d2, r = q1 - p1, q2 - p2, p1 - p2
    a, e, f = d1 @ d1, d2 @ d2, d2 @ r
    eps = 1e-12
    if a <= eps and e <= eps:
        s = t = 0.0
    elif a <= eps:
        s, t = 0.0, min(max(f / e, 0.0), 1.0)
    else:
        c = d1 @ r
        if e <= eps:
            t, s = 0.0, min(max(-c / a, 0.0), 1.0)
        else:
            b = d1 @ d2
            den = a * e - b * b
            s = min(max((b * f - c * e) / den, 0.0), 1.0) if den != 0 else 0.0
            t = (b * s + f) / e
            if t < 0.0:
                t, s = 0.0, min(max(-c / a, 0.0), 1.0)
            elif t > 1.0:
                t, s = 1.0, min(max((b - c) / a, 0.0), 1.0)
    return p1 + d1 * s, p2 + d2 * t


def capsule_separation(body, caps, R, p, i, k):
    """Signed surface distance of proxies i and k."""
    a, b = body[i], body[k]
    ca = [R[a] @ caps[i, 0:3] + p[a], R[a] @ caps[i, 3:6] + p[a]]
    cb = [R[b] @ caps[k, 0:3] + p[b], R[b] @ caps[k, 3:6] + p[b]]
    x, y = segment_closest(ca[0], ca[1], cb[0], cb[1])
    return float(np.linalg.norm(x - y)) - float(caps[i, 6]) - float(caps[k, 6])


@dataclass
class SelfCollision:
    proxy_body: np.ndarray   # [S] int32 body of each capsule proxy
    capsules: np.ndarray     # [S, 7] float32 (p0, p1, radius) in the body frame
    pairs: np.ndarray        # [Q, 2] int32 proxy indices, body of the first < body of the second
    max_self_contacts: int   # contact slots self contacts may take per substep
    dropped_at_rest: list    # proxy pairs excluded because they overlap in the default pose
    unreachable: list        # proxy pairs that never come within reach_margin over the joint box


def _frames_batch(model, Q):
    """body_frames for a batch of joint vectors Q [K, D] -> R [K,B,3,3], p [K,B,3]."""
    K, B = Q.shape[0], model.num_bodies
    R = np.zeros((K, B, 3, 3))
    p = np.zeros((K, B, 3))
    R[:, 0] = np.eye(3)
    for b in range(1, B):
        a = model.parent[b]
        Rj = R[:, a] @ model.joint_rot[b].reshape(3, 3).astype(np.float64)
        p[:, b] = p[:, a] + np.einsum("kij,j->ki", R[:, a], model.joint_pos[b].astype(np.float64))
        j = model.dof[b]
        if j < 0:
            R[:, b] = Rj
            continue
        x, y, z = model.axis[b].astype(np.float64)
        s, c = np.sin(Q[:, j]), np.cos(Q[:, j])
        t = 1.0 - c
        Ra = np.stack([np.stack([t * x * x + c, t * x * y - s * z, t * x * z + s * y], -1),
                       np.stack([t * x * y + s * z, t * y * y + c, t * y * z - s * x], -1),
                       np.stack([t * x * z - s * y, t * y * z + s * x, t * z * z + c], -1)], -2)
        R[:, b] = Rj @ Ra
    return R, p


def _segment_distance_batch(p1, q1, p2, q2):
    """Vectorised segment_closest distance over a leading batch axis."""
    d1, d2, r = q1 - p1, q2 - p2, p1 - p2
    dot = lambda u, v: np.einsum("ki,ki->k", u, v)  # noqa: E731
    a, e, f, c, b = dot(d1, d1), dot(d2, d2), dot(d2, r), dot(d1, r), dot(d1, d2)
    eps = 1e-12
    with np.errstate(divide="ignore", invalid="ignore"):
        den = a * e - b * b
        s = np.where(den != 0, np.clip((b * f - c * e) / den, 0, 1), 0.0)
        s = np.where(a <= eps, 0.0, s)
        t = np.where(e <= eps, 0.0, (b * s + f) / np.where(e <= eps, 1.0, e))
        lo, hi = t < 0, t > 1
        s = np.where(lo & (a > eps), np.clip(-c / np.where(a > eps, a, 1.0), 0, 1), s)
        s = np.where(hi & (a > eps), np.clip((b - c) / np.where(a > eps, a, 1.0), 0, 1), s)
        t = np.clip(t, 0, 1)
        s = np.where((e <= eps) & (a > eps), np.clip(-c / np.where(a > eps, a, 1.0), 0, 1), s)
        t = np.where((a <= eps) & (e > eps), np.clip(f / np.where(e > eps, e, 1.0), 0, 1), t)
    return np.linalg.norm((p1 + d1 * s[:, None]) - (p2 + d2 * t[:, None]), axis=1)


_CACHE = {}


def build_self_collision(model, q_default, max_self_contacts=4, **kw):
    """build_self_collision_uncached, memoised per (model, default pose, options) in this process."""
    key = (model.name, model.num_points, tuple(np.round(np.asarray(q_default, dtype=np.float64), 9)),
           int(max_self_contacts), tuple(sorted(kw.items())))
    if key not in _CACHE:
        _CACHE[key] = build_self_collision_uncached(model, q_default, max_self_contacts, **kw)
    return _CACHE[key]


def build_self_collision_uncached(model, q_default, max_self_contacts=4, rest_margin=0.01, reach_margin=0.02,
                         reach_samples=4096, seed=0):
    """Proxies and the tested pairs of a model; q_default: the default joint angles [D]."""
    body, caps = capsule_proxies(model)
    S = len(body)
    if S > MAX_PROXIES:
        raise ValueError(f"{model.name}: {S} collision shapes exceed {MAX_PROXIES}")
    R, p = body_frames(model, np.asarray(q_default, dtype=np.float64))
    lo = np.clip(model.dof_lower.astype(np.float64), -np.pi, np.pi)
    hi = np.clip(model.dof_upper.astype(np.float64), -np.pi, np.pi)
    Q = np.random.default_rng(seed).uniform(lo, hi, size=(reach_samples, model.num_dofs))
    RK, pK = _frames_batch(model, Q)
    # every proxy's world segment over the sampled poses
    seg = [(np.einsum("kij,j->ki", RK[:, body[i]], caps[i, 0:3].astype(np.float64)) + pK[:, body[i]],
            np.einsum("kij,j->ki", RK[:, body[i]], caps[i, 3:6].astype(np.float64)) + pK[:, body[i]])
           for i in range(S)]
    pairs, dropped, unreachable = [], [], []
    for i in range(S):
        for k in range(S):
            a, b = int(body[i]), int(body[k])
            if not a < b or model.parent[b] == a:  # same link, or joined by a joint
                continue
            if capsule_separation(body, caps, R, p, i, k) < rest_margin:
                dropped.append((i, k))
                continue
            dist = _segment_distance_batch(seg[i][0], seg[i][1], seg[k][0], seg[k][1])
            if (dist - caps[i, 6] - caps[k, 6]).min() >= reach_margin:
                unreachable.append((i, k))
                continue
            pairs.append((i, k))
    if len(pairs) > MAX_PAIRS:
        raise ValueError(f"{model.name}: {len(pairs)} self-collision pairs exceed {MAX_PAIRS}")
    return SelfCollision(body, caps, np.array(pairs, dtype=np.int32).reshape(-1, 2), int(max_self_contacts),
                         dropped, unreachable)
