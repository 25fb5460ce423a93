"""PGS convergence experiment on the oracle copy written by patch.py (not product code): N envs
under random PD gaits, every substep also solved with 200 cold sweeps; prints the mean
constraint-velocity and impulse error of each sweep / warm-start setting against it."""
import ctypes as C, sys, os, time
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
sys.path[:0] = [os.path.join(ROOT, d) for d in ('unitree-rl-gym_amd', 'tests', 'oracle')]
from hostspec import make_spec
from leggedsim import cabi
lib = cabi.load_oracle(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libexp.so'))
lib.exp_set.argtypes = [C.c_int] * 4
lib.exp_stats.argtypes = [C.c_void_p]

def run(task, N, steps, cold, warm_sw, warm, persist, ref=0, seed=0, act_scale=0.5, verbose=False):
    s = make_spec(task)
    if task in ('h1', 'g1', 'h1_2') and s.self_collision is not None:
        import bridge
        bridge.set_self_collision(lib, s.self_collision)
    lib.orc_set_factor_chain(0)
    lib.exp_alloc(N)
    lib.exp_set(cold, warm_sw, warm, ref)
    rng = np.random.default_rng(seed)
    D = s.num_dof
    B = s.num_bodies
    z0 = float(s.base_init_state[2])
    def init(root, dofs, ids):
        for e in ids:
            root[e] = 0; root[e, 2] = z0; root[e, 6] = 1
            root[e, 7:13] = rng.uniform(-0.5, 0.5, 6)
            dofs.reshape(N, D, 2)[e, :, 0] = s.default_dof_pos[0] * rng.uniform(0.5, 1.5, D)
            dofs.reshape(N, D, 2)[e, :, 1] = 0
            lib.exp_clear_one(int(e))
    root = np.zeros((N, 13), np.float32); dofs = np.zeros((N * D, 2), np.float32)
    init(root, dofs, range(N))
    mh = cabi.ModelHandle(s.model)
    cf = np.zeros((N * B, 3), np.float32)
    fr = np.full(N, 1.0, np.float32)
    a = np.zeros((N, D), np.float32)
    kp, kd, lim, d0 = s.p_gains, s.d_gains, s.torque_limits, s.default_dof_pos[0]
    p = lambda x: x.ctypes.data
    dec = s.cfg.control.decimation
    lib.exp_reset_stats()
    falls = 0
    for t in range(steps):
        a = (0.9 * a + 0.45 * rng.normal(0, act_scale, (N, D))).astype(np.float32)
        if not persist:
            lib.exp_clear_ws()
        for k in range(dec):
            q = dofs[:, 0].reshape(N, D); qd = dofs[:, 1].reshape(N, D)
            tau = np.clip(kp * (0.25 * a + d0 - q) - kd * qd, -lim, lim).astype(np.float32)
            lib.orc_simulate(C.byref(mh.desc), C.byref(s.sim_params), N, p(root), p(dofs), p(tau), p(cf), None, None, p(fr))
        # fallen: base low or tilted -> reset
        up = 1 - 2 * (root[:, 3] ** 2 + root[:, 4] ** 2)
        bad = np.where((up < 0.5) | (root[:, 2] < 0.5 * z0) | ~np.isfinite(root).all(1))[0]
        falls += len(bad)
        init(root, dofs, bad)
    out = np.zeros(8)
    lib.exp_stats(out.ctypes.data)
    n = max(out[6], 1)
    return dict(v_rms=out[0] / n, v_max=out[1] / n, lam_err=out[2] / n, lam_mag=out[3] / n, energy=out[4] / n,
                frac_vmax_gt_1cm=out[5] / n, sweeps=out[7], falls=falls, root=root.copy())

if __name__ == '__main__':
    task = sys.argv[1] if len(sys.argv) > 1 else 'go2'
    N, steps = int(sys.argv[2]) if len(sys.argv) > 2 else 256, int(sys.argv[3]) if len(sys.argv) > 3 else 100
    for cold, wsw, warm, persist in [(8, 8, 0, 0), (4, 4, 0, 0), (6, 6, 0, 0), (8, 4, 1, 0), (8, 3, 1, 0), (8, 4, 1, 1), (4, 4, 1, 1), (8, 2, 1, 1), (3, 3, 1, 1), (16, 16, 0, 0)]:
        t0 = time.time()
        r = run(task, N, steps, cold, wsw, warm, persist, ref=200)
        print(f"cold={cold:2d} warm_sw={wsw} warm={warm} persist={persist}: sweeps/solve {r['sweeps']:.2f}  v_rms {r['v_rms']:.2e} v_max {r['v_max']:.2e} "
              f"lam_err/lam {r['lam_err']/max(r['lam_mag'],1e-12):.3e} energy {r['energy']:.2e} P(vmax>1cm/s) {r['frac_vmax_gt_1cm']:.3f} falls {r['falls']}  ({time.time()-t0:.1f}s)", flush=True)
