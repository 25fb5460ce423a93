"""Debug: one physics substep (lgs_simulate) vs orc_simulate; per-env mismatch report.
usage: python tools/dbg_substep.py [task] [n]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from leggedsim import cabi  # noqa: E402
import bridge  # noqa: E402


def main(task="h1_2", n=512):
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name=task, args=args)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(30):
        env.step(0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g))
    tau = (5.0 * torch.randn(n, env.num_dof, device="cuda", generator=g)).contiguous()
    snap = bridge.snapshot(env)
    env.sim.simulate(tau)
    torch.cuda.synchronize()
    lib = bridge.ensure_built()
    mh = cabi.ModelHandle(env.model)
    root, dofs = snap["root"].copy(), snap["dofs"].copy()
    cf, rbs = snap["cforce"].copy(), snap["rbs"].copy()
    t = tau.cpu().numpy()
    p = lambda a: a.ctypes.data  # noqa: E731
    lib.orc_simulate(C.byref(mh.desc), C.byref(env._lgs_params), n, p(root), p(dofs), p(t), p(cf), p(rbs),
                     p(snap["added_mass"]), p(snap["friction"]))
    groot = env.root_states.cpu().numpy()
    gdofs = env.dof_state.cpu().numpy()
    gcf = env._contact_forces.cpu().numpy().reshape(n, -1, 3)
    cf = cf.reshape(n, -1, 3)
    dr = np.abs(groot - root).max(axis=1)
    dd = np.abs(gdofs - dofs).reshape(n, -1).max(axis=1)
    bad = np.where((dr > 1e-3) | (dd > 1e-3))[0]
    ncont_ref = (np.abs(cf).sum(axis=2) > 0).sum(axis=1)
    ncont_gpu = (np.abs(gcf).sum(axis=2) > 0).sum(axis=1)
    print(f"{task}: {len(bad)}/{n} envs differ; max root diff {dr.max():.3e} dof diff {dd.max():.3e}")
    print("contact bodies (ref) histogram all:", np.bincount(ncont_ref))
    if len(bad):
        print("contact bodies (ref) histogram bad:", np.bincount(ncont_ref[bad]))
        # limit activity: dofs near limits
        lo, hi = env.model.dof_lower, env.model.dof_upper
        q = snap["dofs"].reshape(n, -1, 2)[..., 0]
        nlim = ((q < lo + 0.05) | (q > hi - 0.05)).sum(axis=1)
        print("near-limit dofs all:", np.bincount(nlim), " bad:", np.bincount(nlim[bad]))
        for e in bad[:3]:
            print(f"env {e}: root diff {dr[e]:.3e} dof diff {dd[e]:.3e}")
            print("  cf ref:", np.round(cf[e], 2).tolist())
            print("  cf gpu:", np.round(gcf[e], 2).tolist())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "h1_2", int(sys.argv[2]) if len(sys.argv) > 2 else 512)
