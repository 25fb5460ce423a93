"""URDF -> articulated-model loader with IsaacGym asset-import semantics.

This replaces the model side of ``gym.load_asset`` as the reference calls it at
``legged_gym/envs/base/legged_robot.py:294-328`` with the AssetOptions of
``legged_robot_config.py:120-144``:

* ``collapse_fixed_joints=True``: a child attached by a ``fixed`` joint is merged
  into its parent (mass, centre of mass, inertia and collision shapes) unless the
  joint carries ``dont_collapse="true"``; then it stays a separate rigid body
  with a 0-DOF joint (Go2 feet / head, ``go2.urdf``).
* bodies and DOFs are numbered depth-first, children in URDF joint order
  (this reproduces the body indices the reference looks up with
  ``find_actor_rigid_body_handle``, e.g. Go2 feet 6/10/14/18).
* ``replace_cylinder_with_capsule=True``: a collision cylinder becomes a capsule
  of the same radius whose segment spans the cylinder length.
* mesh colliders are reduced to a bounded set of convex-hull support points
  (plane/heightfield contact only ever needs the extreme points).

Everything here runs once at env creation on the host; the result is packed
into flat arrays by :mod:`leggedsim.model` for the HIP simulator.
"""
from __future__ import annotations

import math
import os
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np


def rpy_to_mat(rpy):
    """URDF fixed-axis roll/pitch/yaw -> rotation matrix (Rz*Ry*Rx)."""
    r, p, y = rpy
    cr, sr = math.cos(r), math.sin(r)
    cp, sp = math.cos(p), math.sin(p)
    cy, sy = math.cos(y), math.sin(y)
    rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return rz @ ry @ rx


def _vec(s, n=3, default=0.0):
    if s is None:
        return np.full(n, default, dtype=np.float64)
    return np.array([float(x) for x in s.split()], dtype=np.float64)


@dataclass
class Shape:
    kind: str                 # 'sphere' | 'capsule' | 'box' | 'points'
    rot: np.ndarray           # 3x3, shape frame in body frame
    pos: np.ndarray           # 3
    radius: float = 0.0
    half_length: float = 0.0  # capsule half segment length (along shape z)
    half_extents: np.ndarray = None  # box
    points: np.ndarray = None  # (k,3) hull support points in shape frame
    link: str = ""            # URDF link the shape was declared on (kept through fixed-joint collapse)


@dataclass
class Link:
    name: str
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    inertia: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))  # about com, link frame
    shapes: list = field(default_factory=list)


@dataclass
class Joint:
    name: str
    jtype: str
    parent: str
    child: str
    rot: np.ndarray
    pos: np.ndarray
    axis: np.ndarray
    lower: float = 0.0
    upper: float = 0.0
    effort: float = 0.0
    velocity: float = 0.0
    dont_collapse: bool = False


def read_stl(path):
    """Vertices (n,3) of a binary or ASCII STL file."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:5] == b"solid" and b"facet" in data[:512]:
        verts = []
        for line in data.decode(errors="ignore").splitlines():
            line = line.strip()
            if line.startswith("vertex"):
                verts.append([float(x) for x in line.split()[1:4]])
        return np.unique(np.array(verts, dtype=np.float64), axis=0)
    ntri = struct.unpack("<I", data[80:84])[0]
    rec = np.frombuffer(data[84:84 + ntri * 50], dtype=np.dtype([
        ("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    return np.unique(rec["v"].reshape(-1, 3).astype(np.float64), axis=0)


def hull_support_points(verts, k):
    """Reduce a vertex cloud to <= k convex-hull points by farthest-point sampling,
    seeded with the 6 axis extremes so that the lowest point in any near-upright
    pose is always kept."""
    try:
        from scipy.spatial import ConvexHull
        hv = verts[ConvexHull(verts).vertices]
    except Exception:  # degenerate cloud
        hv = verts
    if len(hv) <= k:
        return hv
    chosen = []
    for ax in range(3):
        chosen.append(int(np.argmin(hv[:, ax])))
        chosen.append(int(np.argmax(hv[:, ax])))
    chosen = list(dict.fromkeys(chosen))
    d = np.min(np.linalg.norm(hv[:, None, :] - hv[chosen][None], axis=-1), axis=1)
    while len(chosen) < k:
        i = int(np.argmax(d))
        chosen.append(i)
        d = np.minimum(d, np.linalg.norm(hv - hv[i], axis=-1))
    return hv[chosen]


def parse_urdf(path, mesh_points=16):
    root = ET.parse(path).getroot()
    base_dir = os.path.dirname(os.path.abspath(path))
    links = {}
    for l in root.findall("link"):
        link = Link(l.get("name"))
        inn = l.find("inertial")
        if inn is not None:
            o = inn.find("origin")
            rot = rpy_to_mat(_vec(o.get("rpy") if o is not None else None))
            link.com = _vec(o.get("xyz") if o is not None else None)
            link.mass = float(inn.find("mass").get("value"))
            ia = inn.find("inertia").attrib
            ixx, iyy, izz = float(ia["ixx"]), float(ia["iyy"]), float(ia["izz"])
            ixy, ixz, iyz = float(ia.get("ixy", 0)), float(ia.get("ixz", 0)), float(ia.get("iyz", 0))
            ii = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])
            link.inertia = rot @ ii @ rot.T
        for c in l.findall("collision"):
            o = c.find("origin")
            rot = rpy_to_mat(_vec(o.get("rpy") if o is not None else None))
            pos = _vec(o.get("xyz") if o is not None else None)
            g = c.find("geometry")[0]
            if g.tag == "sphere":
                link.shapes.append(Shape("sphere", rot, pos, radius=float(g.get("radius")), link=link.name))
            elif g.tag == "cylinder":
                link.shapes.append(Shape("capsule", rot, pos, radius=float(g.get("radius")),
                                         half_length=0.5 * float(g.get("length")), link=link.name))
            elif g.tag == "box":
                link.shapes.append(Shape("box", rot, pos, half_extents=0.5 * _vec(g.get("size")), link=link.name))
            elif g.tag == "mesh":
                fn = g.get("filename")
                if fn.startswith("package://"):
                    fn = fn.split("/", 3)[-1]
                mp = os.path.normpath(os.path.join(base_dir, fn))
                if not os.path.exists(mp):
                    continue  # e.g. blobs listed in the reference's .MISSING_LARGE_BLOBS
                scale = _vec(g.get("scale"), default=1.0) if g.get("scale") else np.ones(3)
                pts = hull_support_points(read_stl(mp) * scale, mesh_points)
                link.shapes.append(Shape("points", rot, pos, points=pts, link=link.name))
        links[link.name] = link
    joints = []
    for j in root.findall("joint"):
        o = j.find("origin")
        a = j.find("axis")
        lim = j.find("limit")
        jt = Joint(j.get("name"), j.get("type"), j.find("parent").get("link"), j.find("child").get("link"),
                   rpy_to_mat(_vec(o.get("rpy") if o is not None else None)),
                   _vec(o.get("xyz") if o is not None else None),
                   _vec(a.get("xyz") if a is not None else "1 0 0"),
                   dont_collapse=(j.get("dont_collapse", "false").lower() == "true"))
        if jt.jtype == "continuous":
            jt.jtype = "revolute"
            jt.lower, jt.upper = -1e9, 1e9
        if lim is not None:
            jt.lower = float(lim.get("lower", jt.lower))
            jt.upper = float(lim.get("upper", jt.upper))
            jt.effort = float(lim.get("effort", 0.0))
            jt.velocity = float(lim.get("velocity", 0.0))
        n = np.linalg.norm(jt.axis)
        jt.axis = jt.axis / n if n > 0 else np.array([1.0, 0.0, 0.0])
        joints.append(jt)
    return links, joints


def _merge_into(parent: Link, child: Link, rot, pos):
    """Merge ``child`` (whose frame is (rot,pos) in the parent frame) into parent."""
    m1, m2 = parent.mass, child.mass
    c2 = rot @ child.com + pos
    I2 = rot @ child.inertia @ rot.T
    m = m1 + m2
    if m > 0:
        com = (m1 * parent.com + m2 * c2) / m
    else:
        com = parent.com.copy()

    def shift(I, mass, c):
        d = c - com
        return I + mass * (np.dot(d, d) * np.eye(3) - np.outer(d, d))

    parent.inertia = shift(parent.inertia, m1, parent.com) + shift(I2, m2, c2)
    parent.mass, parent.com = m, com
    for s in child.shapes:
        parent.shapes.append(Shape(s.kind, rot @ s.rot, rot @ s.pos + pos, s.radius, s.half_length,
                                   s.half_extents, s.points, s.link))


@dataclass
class Body:
    name: str
    parent: int
    joint_name: str
    joint_type: str        # 'root' | 'revolute' | 'fixed'
    joint_rot: np.ndarray  # parent body frame -> joint frame
    joint_pos: np.ndarray
    axis: np.ndarray
    link: Link
    dof: int = -1


@dataclass
class Articulation:
    bodies: list
    dof_names: list
    dof_lower: np.ndarray
    dof_upper: np.ndarray
    dof_effort: np.ndarray
    dof_velocity: np.ndarray

    @property
    def body_names(self):
        return [b.name for b in self.bodies]


def build_articulation(path, collapse_fixed_joints=True, mesh_points=16):
    links, joints = parse_urdf(path, mesh_points=mesh_points)
    children = {}
    child_set = set()
    for j in joints:
        children.setdefault(j.parent, []).append(j)
        child_set.add(j.child)
    roots = [n for n in links if n not in child_set]
    if len(roots) != 1:
        raise ValueError(f"URDF {path}: expected one root link, found {roots}")
    bodies = []
    dof_names, lo, hi, eff, vel = [], [], [], [], []

    def visit(link_name, body_idx):
        """Attach the subtree below ``link_name`` (already represented by body ``body_idx``)."""
        for j in children.get(link_name, []):
            child = links[j.child]
            if j.jtype == "fixed" and collapse_fixed_joints and not j.dont_collapse:
                # merge child (and, recursively, its collapsed descendants) into body_idx,
                # composing transforms relative to the body frame.
                rot, pos = _collapse_chain(body_idx, link_name, j)
                _merge_into(bodies[body_idx].link, child, rot, pos)
                _visit_collapsed(j.child, body_idx, rot, pos)
                continue
            jt = "revolute" if j.jtype in ("revolute", "continuous") else "fixed"
            if j.jtype == "prismatic":
                raise NotImplementedError("prismatic joints are not used by any registered robot")
            rot, pos = _frame_of(link_name, body_idx)
            b = Body(child.name, body_idx, j.name, jt, rot @ j.rot, rot @ j.pos + pos, j.axis.copy(),
                     Link(child.name, child.mass, child.com.copy(), child.inertia.copy(), list(child.shapes)))
            if jt == "revolute":
                b.dof = len(dof_names)
                dof_names.append(j.name)
                lo.append(j.lower); hi.append(j.upper); eff.append(j.effort); vel.append(j.velocity)
            bodies.append(b)
            _link_frame[child.name] = (len(bodies) - 1, np.eye(3), np.zeros(3))
            visit(child.name, len(bodies) - 1)

    # link name -> (body index, rot, pos) of that link's frame inside its body
    _link_frame = {}

    def _frame_of(link_name, body_idx):
        bi, rot, pos = _link_frame[link_name]
        assert bi == body_idx
        return rot, pos

    def _collapse_chain(body_idx, link_name, j):
        rot, pos = _frame_of(link_name, body_idx)
        return rot @ j.rot, rot @ j.pos + pos

    def _visit_collapsed(link_name, body_idx, rot, pos):
        _link_frame[link_name] = (body_idx, rot, pos)
        visit(link_name, body_idx)

    r = links[roots[0]]
    bodies.append(Body(r.name, -1, "root", "root", np.eye(3), np.zeros(3), np.zeros(3),
                       Link(r.name, r.mass, r.com.copy(), r.inertia.copy(), list(r.shapes))))
    _link_frame[r.name] = (0, np.eye(3), np.zeros(3))
    visit(r.name, 0)
    return Articulation(bodies, dof_names, np.array(lo), np.array(hi), np.array(eff), np.array(vel))
