"""Compile the robot URDFs the registered tasks use into bundled model files.

Reads the reference's robot descriptions (URDF + STL, read-only) and writes
unitree-rl-gym_amd/leggedsim/models/<stem>.npz: the collapsed articulation
(inertias, joint frames, limits) and contact candidate points.  These are
derived data, so the simulator runs where the robot description tree is absent
(e.g. the GPU box).  Re-run after changing urdf.py/model.py:
    python tools/build_models.py [/root/reference/resources/robots]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "unitree-rl-gym_amd"))

from leggedsim.model import MODELS_DIR, load_model  # noqa: E402

ROBOTS = ["go2/urdf/go2.urdf", "g1_description/g1_12dof.urdf", "h1/urdf/h1.urdf", "h1_2/h1_2_12dof.urdf",
          # another robot the reference ships, for the plugin-task test of the build-time shape hook
          "g1_description/g1_23dof.urdf"]


def main(root):
    os.makedirs(MODELS_DIR, exist_ok=True)
    for rel in ROBOTS:
        m = load_model(os.path.join(root, rel))
        out = os.path.join(MODELS_DIR, m.name + ".npz")
        m.save(out)
        print(f"{rel}: {m.num_bodies} bodies, {m.num_dofs} dofs, {m.num_points} contact points -> {out}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/resources/robots")
