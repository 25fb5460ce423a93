"""The self-collision proxies of the humanoid tasks per body (leggedsim/selfcollision.py: one
capsule per URDF collision shape, a fixed-joint-collapsed link keeping every shape of the links
merged into it) and the pairs the step tests.  usage: python tools/self_collision_table.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "unitree-rl-gym_amd"), os.path.join(ROOT, "tests")]
from hostspec import make_spec  # noqa: E402

for task in ("h1", "g1", "h1_2"):
    s = make_spec(task)
    sc, m = s.self_collision, s.model
    print(f"{task}: {len(sc.proxy_body)} capsule proxies on {m.num_bodies} bodies, {len(sc.pairs)} tested pairs "
          f"({len(sc.dropped_at_rest)} overlapping at rest, {len(sc.unreachable)} unreachable dropped), "
          f"max {sc.max_self_contacts} self contacts per substep")
    for b in range(m.num_bodies):
        k = np.where(sc.proxy_body == b)[0]
        if not len(k):
            continue
        npair = int(np.isin(sc.pairs, k).any(axis=1).sum())
        lens = [float(np.linalg.norm(sc.capsules[i, 3:6] - sc.capsules[i, 0:3])) for i in k]
        print(f"  {m.body_names[b]:24s} {len(k):2d} capsules (radius {min(sc.capsules[k, 6]):.3f}-{max(sc.capsules[k, 6]):.3f} m, "
              f"segment {min(lens):.3f}-{max(lens):.3f} m) in {npair} pairs")
