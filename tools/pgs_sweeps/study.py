"""PGS sweep-count study: convergence of the contact solve against sweeps,
on the CPU oracle's arithmetic (make_exp.py's instrumented copy; the HIP kernel is bit-exact
with the oracle, so these are the kernel's numbers).

  python tools/pgs_sweeps/study.py curves   [tasks] -> error vs sweeps k = 1..16 per solver variant,
        on states of a random-PD-gait rollout integrated with the converged (200-sweep) solve
  python tools/pgs_sweeps/study.py poses             -> the same on the contact-pose fixtures
        (tests/golden/contact_poses.npz: humanoids kneeling / sitting, substeps 1..8 of a step)
  python tools/pgs_sweeps/study.py kneel             -> the H1_2 kneel impact at -0.2 m/s: knee
        force per substep for 4 / 5 / 6 / 8 / 200 sweeps (test_gpu_contact_slots' case)
  python tools/pgs_sweeps/study.py closed [tasks]    -> rollouts integrated with k sweeps: the
        error of the iterate actually used, base height, falls

Writes JSON + a text table into profiles/round6/pgs_sweeps/ (or $OUT)."""
import copy
import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("unitree-rl-gym_amd", "tests", "oracle")]
OUT = os.environ.get("OUT", os.path.join(ROOT, "profiles", "round6", "pgs_sweeps"))

KMAX = 24
NM = 12
METRICS = ["solves", "lam_rel_normal", "lam_rel_friction", "v_err_max", "p_v_err_gt_1cm", "energy_rel",
           "total_normal_rel", "p_energy_rel_gt_5pct", "normal_v_residual_max", "solves_loaded", "sweeps_used",
           "p_at_cap"]
VARIANTS = {0: "pgs", 1: "pgs_symmetric", 2: "block3", 3: "block3_symmetric"}
# grouped sweeps (make_exp.py variants 8 / 9): a body's ground contacts' normals solved jointly, or
# only visited together; selected with VARIANTS_SEL=0,8,9
EXTRA_VARIANTS = {8: "group_normal_lcp", 9: "group_order"}
if os.environ.get("VARIANTS_SEL"):
    VARIANTS = {int(v): {**VARIANTS, **EXTRA_VARIANTS}[int(v)] for v in os.environ["VARIANTS_SEL"].split(",")}


def build():
    subprocess.check_call([sys.executable, os.path.join(HERE, "make_exp.py")])
    so = os.path.join(HERE, "libexp_sweeps.so")
    subprocess.check_call(["gcc", "-O3", "-march=native", "-ffp-contract=off", "-fPIC", "-fopenmp", "-std=gnu11",
                           "-shared", "-o", so, os.path.join(HERE, "exp_sweeps.c"), "-lm"])
    from leggedsim import cabi
    lib = cabi.load_oracle(so)
    lib.exp_set.argtypes = [C.c_int] * 4
    lib.exp_stats.argtypes = [C.c_void_p]
    lib.exp_tol.argtypes = [C.c_float]
    return lib


def stats(lib):
    out = np.zeros((KMAX + 1, NM))
    lib.exp_stats(out.ctypes.data)
    res = {}
    for k in range(0, KMAX + 1):
        n, nl = out[k, 0], out[k, 9]
        if n == 0:
            continue
        res[k] = {"solves": int(n), "solves_loaded": int(nl)}
        for m in (3, 4, 8, 10, 11):
            res[k][METRICS[m]] = out[k, m] / n
        for m in (1, 2, 5, 6, 7):
            res[k][METRICS[m]] = out[k, m] / max(nl, 1)
    return res


def gait(lib, task, N, steps, seed=0, act_scale=0.5, sweeps=None):
    """orc_simulate under random PD gaits (drive.py's), fallen envs re-initialised."""
    from hostspec import make_spec
    from leggedsim import cabi
    import bridge
    s = make_spec(task)
    bridge.set_self_collision(lib, s.self_collision)
    lib.orc_set_factor_chain(0)
    sp = copy.copy(s.sim_params)
    if sweeps is not None:
        sp.solver_iterations = sweeps
    rng = np.random.default_rng(seed)
    D, B = s.num_dof, s.num_bodies
    z0 = float(s.base_init_state[2])

    def init(root, dofs, ids):
        for e in ids:
            root[e] = 0
            root[e, 2] = z0
            root[e, 6] = 1
            root[e, 7:13] = rng.uniform(-0.5, 0.5, 6)
            dofs.reshape(N, D, 2)[e, :, 0] = s.default_dof_pos[0] * rng.uniform(0.5, 1.5, D)
            dofs.reshape(N, D, 2)[e, :, 1] = 0
    root = np.zeros((N, 13), np.float32)
    dofs = np.zeros((N * D, 2), np.float32)
    init(root, dofs, range(N))
    mh = cabi.ModelHandle(s.model)
    cf = np.zeros((N * B, 3), np.float32)
    fr = np.full(N, 1.0, np.float32)
    a = np.zeros((N, D), np.float32)
    kp, kd, lim, d0 = s.p_gains, s.d_gains, s.torque_limits, s.default_dof_pos[0]
    dec = s.cfg.control.decimation
    falls, heights = 0, []
    for t in range(steps):
        a = (0.9 * a + 0.45 * rng.normal(0, act_scale, (N, D))).astype(np.float32)
        for _ in range(dec):
            q = dofs[:, 0].reshape(N, D)
            qd = dofs[:, 1].reshape(N, D)
            tau = np.clip(kp * (0.25 * a + d0 - q) - kd * qd, -lim, lim).astype(np.float32)
            lib.orc_simulate(C.byref(mh.desc), C.byref(sp), N, root.ctypes.data, dofs.ctypes.data, tau.ctypes.data,
                             cf.ctypes.data, None, None, fr.ctypes.data)
        up = 1 - 2 * (root[:, 3] ** 2 + root[:, 4] ** 2)
        heights.append(float(root[:, 2].mean()))
        bad = np.where((up < 0.5) | (root[:, 2] < 0.5 * z0) | ~np.isfinite(root).all(1))[0]
        falls += len(bad)
        init(root, dofs, bad)
    return {"falls_per_env_step": falls / (N * steps), "mean_base_height": float(np.mean(heights[steps // 2:]))}


def curves(lib, tasks, N=256, steps=60):
    res = {}
    for task in tasks:
        res[task] = {}
        for v, name in VARIANTS.items():
            t0 = time.time()
            lib.exp_set(v, 16, 200, 1)
            lib.exp_reset()
            gait(lib, task, N, steps, seed=1)
            res[task][name] = stats(lib)
            print(f"curves {task} {name}: {time.time() - t0:.1f}s", flush=True)
    return res


def poses(lib):
    """The contact-pose fixtures, one control step of 8 substeps each, pressed at -0.2 m/s."""
    from hostspec import host_buffers, make_spec
    import bridge
    z = np.load(os.path.join(ROOT, "tests", "golden", "contact_poses.npz"))
    res = {}
    for v, name in VARIANTS.items():
        lib.exp_set(v, 16, 200, 1)
        lib.exp_reset()
        for task in ("h1", "g1", "h1_2"):
            s = make_spec(task)
            for pose in ("kneel", "sit"):
                key = f"{task}_{pose}_root"
                if key not in z:
                    continue
                N = 2
                b = host_buffers(s, N)
                b["root"][:] = z[key]
                b["root"][:, 9] = -0.2
                q = z[f"{task}_{pose}_q"]
                b["dofs"].reshape(N, -1, 2)[:, :, 0] = q
                b["actions"][:] = (q - s.default_dof_pos[0]) / s.cfg.control.action_scale
                T = copy.copy(s.task)
                T.decimation, T.push_robots, T.add_noise = 8, 0, 0
                bridge.step_raw(s.model, s.sim_params, T, N, b, 0, lib=lib, self_collision=s.self_collision)
        res[name] = stats(lib)
    return res


def kneel(lib, sweeps_list=(4, 5, 6, 8, 12, 200)):
    """H1_2 kneeling, pressed into the ground at -0.2 m/s: knee contact force after 1..8
    substeps (test_gpu_contact_slots: 200 sweeps give 318 N, shipped 8 sweeps 304 N)."""
    from hostspec import host_buffers, make_spec
    from leggedsim import cabi
    import bridge
    z = np.load(os.path.join(ROOT, "tests", "golden", "contact_poses.npz"))
    res = {}
    for task in ("h1_2", "h1", "g1"):
        s = make_spec(task)
        knees = [i for i, n in enumerate(s.model.body_names) if "knee" in n]
        res[task] = {}
        for v, name in ((0, "pgs"), (2, "block3")):
            for sw in sweeps_list:
                lib.exp_set(v, sw, 0, 0)
                forces, zs = [], []
                for dec in range(1, 9):
                    sp = cabi.sim_params_from_cfg(s.cfg.sim, s.cfg.asset, max_contacts=s.sim_params.max_contacts,
                                                  max_rows=s.sim_params.max_rows, solver_iterations=sw,
                                                  ground_friction=s.sim_params.ground_friction)
                    N = 2
                    b = host_buffers(s, N)
                    b["root"][:] = z[f"{task}_kneel_root"]
                    b["root"][:, 9] = -0.2
                    q = z[f"{task}_kneel_q"]
                    b["dofs"].reshape(N, -1, 2)[:, :, 0] = q
                    b["actions"][:] = (q - s.default_dof_pos[0]) / s.cfg.control.action_scale
                    T = copy.copy(s.task)
                    T.decimation, T.push_robots, T.add_noise = dec, 0, 0
                    bridge.step_raw(s.model, sp, T, N, b, 0, lib=lib, self_collision=s.self_collision)
                    cf = b["cforce"].reshape(N, -1, 3)
                    forces.append(float(np.linalg.norm(cf[0, knees], axis=1).sum()))
                    zs.append(float(b["root"][0, 2]))
                res[task][f"{name}_{sw}"] = {"knee_force_N_per_substep": [round(f, 2) for f in forces],
                                              "base_z_per_substep": [round(x, 5) for x in zs]}
                print(f"kneel {task} {name} {sw:3d} sweeps: knee |F| " + " ".join(f"{f:7.1f}" for f in forces), flush=True)
    return res


def closed(lib, tasks, sweeps_list=(4, 5, 6, 8, 16), N=256, steps=100):
    res = {}
    for task in tasks:
        res[task] = {}
        for v, name in ((0, "pgs"), (2, "block3")):
            for sw in sweeps_list:
                lib.exp_set(v, sw, 200, 0)
                lib.exp_reset()
                g = gait(lib, task, N, steps, seed=2, sweeps=sw)
                st = stats(lib)
                g.update({"at_used_count": st.get(sw, {})})
                res[task][f"{name}_{sw}"] = g
                e = g["at_used_count"]
                print(f"closed {task} {name} {sw:2d}: energy_rel {e.get('energy_rel', 0):.3e} lam_n {e.get('lam_rel_normal', 0):.3e} "
                      f"vmax {e.get('v_err_max', 0):.2e} falls {g['falls_per_env_step']:.4f} z {g['mean_base_height']:.4f}",
                      flush=True)
    return res


def adaptive(lib, tasks, tols=(3e-3, 1e-3, 3e-4, 1e-4), N=256, steps=100, cap=8):
    """Variant 4: sweeps stop once a sweep's largest row residual |dlam_r| A_rr <= tol (at most
    `cap`): closed-loop rollouts, the stopped iterate's error and the sweeps it used."""
    res = {}
    for task in tasks:
        res[task] = {}
        for tol in tols:
            lib.exp_set(4, cap, 200, 0)
            lib.exp_tol(tol)
            lib.exp_reset()
            g = gait(lib, task, N, steps, seed=2, sweeps=cap)
            st = stats(lib)
            g.update({"stopped": st.get(0, {})})
            res[task][f"tol_{tol:g}"] = g
            e = g["stopped"]
            print(f"adaptive {task} tol {tol:g}: sweeps {e.get('sweeps_used', 0):.2f} (at cap {e.get('p_at_cap', 0):.3f}) "
                  f"energy_rel {e.get('energy_rel', 0):.3e} vmax {e.get('v_err_max', 0):.2e} "
                  f"P(v>1cm) {e.get('p_v_err_gt_1cm', 0):.3f} falls {g['falls_per_env_step']:.4f}", flush=True)
    return res


def table(curv, ks=(1, 2, 3, 4, 5, 6, 8, 10, 12, 16)):
    lines = []
    for task, byv in curv.items():
        lines.append(f"== {task}")
        for m in ("energy_rel", "lam_rel_normal", "lam_rel_friction", "total_normal_rel", "v_err_max", "p_v_err_gt_1cm",
                  "p_energy_rel_gt_5pct"):
            lines.append(f"  {m}")
            for name, st in byv.items():
                row = " ".join(f"{st[k][m]:9.2e}" if k in st else "        -" for k in ks)
                lines.append(f"    {name:17s} {row}")
        lines.append("    k =               " + " ".join(f"{k:9d}" for k in ks))
    return "\n".join(lines)


if __name__ == "__main__":
    what = sys.argv[1]
    tasks = sys.argv[2].split(",") if len(sys.argv) > 2 else ["go2", "h1", "h1_2", "g1"]
    os.makedirs(OUT, exist_ok=True)
    lib = build()
    if what == "curves":
        r = curves(lib, tasks)
        txt = table(r)
    elif what == "poses":
        r = poses(lib)
        txt = table({"contact_poses": r})
    elif what == "kneel":
        r = kneel(lib)
        txt = json.dumps(r, indent=1)
    elif what == "closed":
        r = closed(lib, tasks)
        txt = json.dumps(r, indent=1)
    elif what == "adaptive":
        r = adaptive(lib, tasks)
        txt = json.dumps(r, indent=1)
    else:
        raise SystemExit(__doc__)
    tag = what + ("_" + "_".join(tasks) if what in ("curves", "closed", "adaptive") else "")
    with open(os.path.join(OUT, tag + ".json"), "w") as f:
        json.dump(r, f, indent=1)
    with open(os.path.join(OUT, tag + ".txt"), "w") as f:
        f.write(txt + "\n")
    print(txt)
