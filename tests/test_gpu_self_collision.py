"""HIP == oracle for self-collision (create_actor's self_collisions filter, reference
legged_robot.py:373-374), on poses where the humanoids' legs touch: one physics substep
(gym.simulate) from crossed-leg states in the air matches the CPU oracle bit for bit and the
self contacts really fire (equal and opposite forces on the touching links, nothing from the
ground); then fused control steps from those states match the oracle bit for bit."""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
import bridge  # noqa: E402
from leggedsim import cabi  # noqa: E402
from test_gpu_parity import STATE, POST, assert_exact, env_arrays, make, writes_body_states  # noqa: E402
from test_self_collision import crossed_pose  # noqa: E402


@pytest.mark.parametrize("task", ["h1", "g1", "h1_2"])
def test_self_contact_step_matches_oracle_bitwise(task):
    env = make(task, 256)
    env.reset()
    sc = env.self_collision
    assert sc is not None and len(sc.pairs) > 0
    q, pair, _ = crossed_pose(env.model, sc, env.default_dof_pos.cpu().numpy())
    i, k = sc.pairs[pair]
    a, b = int(sc.proxy_body[i]), int(sc.proxy_body[k])
    n, D = env.num_envs, env.num_dof
    gen = torch.Generator(device="cuda").manual_seed(7)
    # every env: the crossed pose +- 5 mrad, in the air (2.5 m up), at rest
    qs = torch.tensor(q, device="cuda").repeat(n, 1) + 0.005 * (2 * torch.rand(n, D, device="cuda", generator=gen) - 1)
    env.dof_state.view(n, D, 2)[:, :, 0] = qs
    env.dof_state.view(n, D, 2)[:, :, 1] = 0.0
    env.root_states[:, 2] = env.env_origins[:, 2] + 2.5
    env.root_states[:, 3:7] = torch.tensor([0.0, 0.0, 0.0, 1.0], device="cuda")
    env.root_states[:, 7:13] = 0.0
    # one substep with zero torque: the contact impulse of the first substep
    tau = torch.zeros(n, D, device="cuda")
    snap = bridge.snapshot(env)
    env.sim.simulate(tau)
    torch.cuda.synchronize()
    lib = bridge.ensure_built()
    bridge.set_env(lib, env)
    root, dofs, cf, rbs = snap["root"].copy(), snap["dofs"].copy(), snap["cforce"].copy(), snap["rbs"].copy()
    P = lambda x: x.ctypes.data  # noqa: E731
    t = tau.cpu().numpy()
    mh = cabi.ModelHandle(env.model)
    lib.orc_simulate(C.byref(mh.desc), C.byref(env._lgs_params), n, P(root), P(dofs), P(t), P(cf), P(rbs),
                     P(snap["added_mass"]), P(snap["friction"]))
    got_cf = env._contact_forces.cpu().numpy()
    np.testing.assert_array_equal(env.root_states.cpu().numpy(), root)
    np.testing.assert_array_equal(env.dof_state.cpu().numpy(), dofs)
    np.testing.assert_array_equal(got_cf, cf)
    cfe = got_cf.reshape(n, -1, 3)
    touching = np.linalg.norm(cfe[:, a], axis=1) > 1.0
    assert touching.mean() > 0.5, f"{task}: self contact in only {touching.sum()}/{n} envs"
    np.testing.assert_array_equal(cfe[touching, a], -cfe[touching, b])
    # internal forces only (no ground under the robot): they sum to zero per env
    np.testing.assert_allclose(cfe.sum(axis=1), 0.0, atol=1e-4 * np.abs(cfe).max())
    for it in range(2):
        snap = bridge.snapshot(env)
        act = torch.zeros(n, env.num_actions, device="cuda")
        act[:] = torch.tensor((q - env.default_dof_pos.cpu().numpy().reshape(-1)) / env.cfg.control.action_scale,
                              device="cuda")  # hold the crossed pose
        ref = bridge.step(env, snap, act.cpu().numpy(), env.common_step_counter)
        env.step(act)
        got = env_arrays(env)
        assert_exact(got, ref, STATE + POST, n, f"{task} self-contact step {it}",
                     skip_body_states=not writes_body_states(env))
    bridge.set_self_collision(bridge.ensure_built(), None)
