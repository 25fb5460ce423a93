"""The kneel / sit pose of tests/golden/contact_poses.npz pressed into the ground at -0.2 m/s on the
oracle, contact force of the knees after 1..8 substeps, per solver setting.  (solver_warm_iterations
existed only in the dropped round-5 warm-start build; on the shipped oracle every row is cold.)"""
import sys, copy
import numpy as np
import os
ROOT = os.path.abspath(os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..'))
sys.path[:0] = [os.path.join(ROOT, d) for d in ('unitree-rl-gym_amd', 'tests', 'oracle')]
from hostspec import make_spec, host_buffers
from leggedsim import cabi
import bridge
lib = bridge.ensure_built()
task = sys.argv[1] if len(sys.argv) > 1 else 'h1_2'
pose = sys.argv[2] if len(sys.argv) > 2 else 'kneel'
s = make_spec(task)
bridge.set_self_collision(lib, s.self_collision)
z = np.load(os.path.join(ROOT, 'tests', 'golden', 'contact_poses.npz'))
names = s.model.body_names
knees = [i for i, n in enumerate(names) if 'knee' in n]
print('knees', knees, 'touching', z[f'{task}_{pose}_touching'])
for warm, cold in ((0, 200), (0, 8), (5, 8), (0, 16), (8, 16), (10, 16)):
    for dec in (1, 2, 3, 4, 5, 6, 7, 8):
        sp = cabi.sim_params_from_cfg(s.cfg.sim, s.cfg.asset, max_contacts=s.sim_params.max_contacts, max_rows=s.sim_params.max_rows, solver_warm_iterations=warm, solver_iterations=cold)
        N = 2
        b = host_buffers(s, N)
        b['root'][:] = z[f'{task}_{pose}_root']
        b['root'][:, 9] = -0.2
        q = z[f'{task}_{pose}_q']
        b['dofs'].reshape(N, -1, 2)[:, :, 0] = q
        a = (q - s.default_dof_pos[0]) / s.cfg.control.action_scale
        b['actions'][:] = a
        T = copy.copy(s.task); T.decimation = dec; T.push_robots = 0; T.add_noise = 0
        bridge.step_raw(s.model, sp, T, N, b, 0, lib=lib, self_collision=s.self_collision)
        cf = b['cforce'].reshape(N, -1, 3)
        print(f'cold={cold} warm={warm} substeps={dec}: knee |F| {np.linalg.norm(cf[0, knees], axis=1)}  pelvis z {b["root"][0,2]:.4f} vz {b["root"][0,9]:.4f}')
