"""Flat, device-ready model blob built from an :class:`Articulation`.

Layout (all little-endian, float32 / int32), mirrored by ``lgs_model_desc`` in
``include/leggedsim.h``.  Bodies are in depth-first order, so every parent index
is smaller than its child's and the subtree of body ``b`` is the contiguous range
``[b, subtree_end[b])``.  That property is what lets the HIP kernel compute
composite inertias / forces with one lane per body and no inter-lane ordering.

Collision geometry is reduced to *contact candidates*: points with a radius in a
body frame.  sphere -> 1 point, capsule -> its 2 segment end points, box -> 8
corners (radius 0), mesh -> hull support points (radius 0).  Against a plane or a
heightfield a convex primitive's deepest point is always one of these.
"""
from __future__ import annotations

import hashlib
import json
import os
from dataclasses import dataclass

import numpy as np

from .urdf import Articulation, build_articulation

MAX_BODIES = 32
MAX_DOFS = 26
MAX_DEPTH = 10


@dataclass
class Model:
    name: str
    body_names: list
    dof_names: list
    parent: np.ndarray        # [B] int32
    dof: np.ndarray           # [B] int32 (-1 root/fixed)
    subtree_end: np.ndarray   # [B] int32
    depth: np.ndarray         # [B] int32
    chain: np.ndarray         # [B, MAX_DEPTH] int32 ancestors root..b, -1 padded
    joint_rot: np.ndarray     # [B, 9] f32
    joint_pos: np.ndarray     # [B, 3]
    axis: np.ndarray          # [B, 3]
    mass: np.ndarray          # [B]
    com: np.ndarray           # [B, 3]
    inertia: np.ndarray       # [B, 6]  Ixx Iyy Izz Ixy Ixz Iyz about com, body frame
    dof_body: np.ndarray      # [D] int32
    dof_lower: np.ndarray     # [D]
    dof_upper: np.ndarray
    dof_effort: np.ndarray
    dof_velocity: np.ndarray
    pt_body: np.ndarray       # [P] int32
    pt_pos: np.ndarray        # [P, 3]
    pt_radius: np.ndarray     # [P]
    pt_shape: np.ndarray = None  # [P] int32 URDF link whose collision shapes the point belongs to

    @property
    def num_bodies(self):
        return len(self.body_names)

    @property
    def num_dofs(self):
        return len(self.dof_names)

    @property
    def num_points(self):
        return int(self.pt_body.shape[0])

    def total_mass(self):
        return float(self.mass.sum())

    # ---- persistence (bundled compiled models travel without the reference tree)
    def save(self, path):
        arrays = {k: getattr(self, k) for k in self.__dataclass_fields__ if isinstance(getattr(self, k), np.ndarray)}
        meta = {"name": self.name, "body_names": self.body_names, "dof_names": self.dof_names}
        np.savez(path, meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), **arrays)

    @staticmethod
    def load(path):
        z = np.load(path, allow_pickle=False)
        meta = json.loads(bytes(z["meta"]).decode())
        kw = {k: z[k] for k in z.files if k != "meta"}
        m = Model(meta["name"], meta["body_names"], meta["dof_names"], **kw)
        if m.pt_shape is None:  # a model saved before shapes were recorded: one shape per body
            m.pt_shape = m.pt_body.copy()
        return m

    def reorder_points(self, first_bodies):
        """Put the contact candidates of ``first_bodies`` (the feet) first: the contact
        kernel fills its slots with the touching candidates in index order, so this is
        the slot priority when more candidates touch than the solver has rows for.

        The feet's candidates are dealt round-robin over the feet (1st of every foot,
        then the 2nd, ...), and each foot's own list starts with its sole points in
        farthest-point order: with two flat soles down and 8 slots, each foot gets 4
        spread-out sole corners (PhysX's convex-vs-plane manifold also keeps at most 4
        points per patch) instead of one foot taking every slot.  A foot with one
        candidate (Go2) keeps the previous order exactly."""
        feet = sorted(set(int(b) for b in first_bodies))
        per_foot = [self._sole_first_order(np.nonzero(self.pt_body == b)[0]) for b in feet]
        head = []
        for k in range(max((len(p) for p in per_foot), default=0)):
            head.extend(int(p[k]) for p in per_foot if k < len(p))
        in_head = np.zeros(len(self.pt_body), bool)
        in_head[head] = True
        order = np.array(head + [i for i in range(len(self.pt_body)) if not in_head[i]], dtype=np.int64)
        self.pt_body = self.pt_body[order].copy()
        self.pt_pos = self.pt_pos[order].copy()
        self.pt_radius = self.pt_radius[order].copy()
        self.pt_shape = self.pt_shape[order].copy()

    def _sole_first_order(self, idx, sole_band=0.005):
        """Indices idx of one body's candidates: the sole (sphere bottoms within
        sole_band of the lowest, body frame) in farthest-point order over x-y, starting
        from the one farthest from the sole's centre; then the rest in their order."""
        if len(idx) <= 1:
            return list(idx)
        bottom = self.pt_pos[idx, 2] - self.pt_radius[idx]
        sole = [int(i) for i, z in zip(idx, bottom) if z <= bottom.min() + sole_band]
        xy = self.pt_pos[sole, :2].astype(np.float64)
        first = int(np.argmax(((xy - xy.mean(0)) ** 2).sum(1)))
        chosen, dist = [first], ((xy - xy[first]) ** 2).sum(1)
        while len(chosen) < len(sole):
            dist[chosen] = -1.0
            nxt = int(np.argmax(dist))  # ties: the lowest index
            chosen.append(nxt)
            dist = np.minimum(dist, ((xy - xy[nxt]) ** 2).sum(1))
        ordered = [sole[c] for c in chosen]
        return ordered + [int(i) for i in idx if int(i) not in set(ordered)]


def _shape_points(s):
    if s.kind == "sphere":
        return [s.pos.copy()], [s.radius]
    if s.kind == "capsule":
        ax = s.rot[:, 2]
        return [s.pos + ax * s.half_length, s.pos - ax * s.half_length], [s.radius, s.radius]
    if s.kind == "box":
        pts = []
        h = s.half_extents
        for sx in (-1, 1):
            for sy in (-1, 1):
                for sz in (-1, 1):
                    pts.append(s.pos + s.rot @ (h * np.array([sx, sy, sz])))
        return pts, [0.0] * 8
    if s.kind == "points":
        return [s.pos + s.rot @ p for p in s.points], [0.0] * len(s.points)
    raise ValueError(s.kind)


def model_from_articulation(name, art: Articulation) -> Model:
    B = len(art.bodies)
    D = len(art.dof_names)
    if B > MAX_BODIES or D > MAX_DOFS:
        raise ValueError(f"{name}: {B} bodies / {D} dofs exceed MAX_BODIES={MAX_BODIES}/MAX_DOFS={MAX_DOFS}")
    parent = np.array([b.parent for b in art.bodies], dtype=np.int32)
    dof = np.array([b.dof for b in art.bodies], dtype=np.int32)
    subtree_end = np.arange(1, B + 1, dtype=np.int32)
    for b in range(B - 1, 0, -1):
        p = parent[b]
        subtree_end[p] = max(subtree_end[p], subtree_end[b])
    depth = np.zeros(B, dtype=np.int32)
    chain = -np.ones((B, MAX_DEPTH), dtype=np.int32)
    for b in range(B):
        c = []
        x = b
        while x >= 0:
            c.append(x)
            x = parent[x]
        c = c[::-1]
        if len(c) > MAX_DEPTH:
            raise ValueError("tree too deep")
        depth[b] = len(c) - 1
        chain[b, :len(c)] = c
    inertia = np.zeros((B, 6))
    for i, b in enumerate(art.bodies):
        I = b.link.inertia
        inertia[i] = [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]
    pb, pp, pr, ps = [], [], [], []
    groups = {}  # (body, URDF link) -> id: the shapes a link declared, after fixed-joint collapse
    for i, b in enumerate(art.bodies):
        for s in b.link.shapes:
            g = groups.setdefault((i, s.link), len(groups))
            pts, rads = _shape_points(s)
            for p, r in zip(pts, rads):
                pb.append(i); pp.append(p); pr.append(r); ps.append(g)
    dof_body = np.zeros(D, dtype=np.int32)
    for i, b in enumerate(art.bodies):
        if b.dof >= 0:
            dof_body[b.dof] = i
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return Model(
        name=name, body_names=art.body_names, dof_names=list(art.dof_names),
        parent=parent, dof=dof, subtree_end=subtree_end, depth=depth, chain=chain,
        joint_rot=f32([b.joint_rot.reshape(9) for b in art.bodies]),
        joint_pos=f32([b.joint_pos for b in art.bodies]),
        axis=f32([b.axis for b in art.bodies]),
        mass=f32([b.link.mass for b in art.bodies]),
        com=f32([b.link.com for b in art.bodies]),
        inertia=f32(inertia),
        dof_body=dof_body,
        dof_lower=f32(art.dof_lower), dof_upper=f32(art.dof_upper),
        dof_effort=f32(art.dof_effort), dof_velocity=f32(art.dof_velocity),
        pt_body=np.array(pb, dtype=np.int32).reshape(-1),
        pt_pos=f32(np.array(pp).reshape(-1, 3)),
        pt_radius=f32(pr),
        pt_shape=np.array(ps, dtype=np.int32).reshape(-1),
    )


MODELS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "models")


def load_model(asset_file, collapse_fixed_joints=True):
    """Build the model for ``cfg.asset.file``.

    The URDF is parsed when present (``collapse_fixed_joints`` honoured).  Otherwise
    (e.g. on a GPU box where the robot description tree is absent) the bundled
    model compiled from the same URDF by ``tools/build_models.py`` is used.
    """
    stem = os.path.splitext(os.path.basename(asset_file))[0]
    if os.path.exists(asset_file):
        art = build_articulation(asset_file, collapse_fixed_joints=collapse_fixed_joints)
        return model_from_articulation(stem, art)
    bundled = os.path.join(MODELS_DIR, stem + ".npz")
    if os.path.exists(bundled) and collapse_fixed_joints:
        return Model.load(bundled)
    raise FileNotFoundError(f"asset {asset_file} not found and no bundled model '{stem}' in {MODELS_DIR}")
