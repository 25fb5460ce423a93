"""The CPU oracle's post-physics restatement vs golden vectors produced by the
REFERENCE's own code (oracle/gen_golden.py): PD torques, base-frame quantities,
commands (resampling + heading), termination, every reward term, reset, push,
observation noise and clipping, episode bookkeeping.  Tolerance 1e-5 (fp32)."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import GOLDEN
from hostspec import host_buffers, make_spec
import bridge
from leggedsim import cabi

TASKS = ["go2", "h1", "g1", "h1_2"]
TOL = dict(rtol=1e-5, atol=1e-5)


def load(task):
    return dict(np.load(os.path.join(GOLDEN, f"post_physics_{task}.npz")))


@pytest.mark.parametrize("task", TASKS)
def test_derived_constants_match_reference(task):
    g = load(task)
    s = make_spec(task)
    np.testing.assert_allclose(s.p_gains, g["ref_p_gains"])
    np.testing.assert_allclose(s.d_gains, g["ref_d_gains"])
    np.testing.assert_allclose(s.default_dof_pos, g["ref_default_dof_pos"])
    np.testing.assert_allclose(s.dof_pos_limits, g["ref_dof_pos_limits"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(s.noise_scale_vec, g["ref_noise_vec"])
    np.testing.assert_array_equal(s.feet_indices, g["ref_feet_indices"])
    np.testing.assert_array_equal(s.penalised_contact_indices, g["ref_penalised"])
    np.testing.assert_array_equal(s.termination_contact_indices, g["ref_termination"])
    assert list(s.sum_names) == list(g["ref_reward_names"])  # alphabetical, zeros dropped
    np.testing.assert_allclose([s.reward_scales[k] for k in s.sum_names], g["ref_reward_scales"], rtol=1e-12)


@pytest.mark.parametrize("task", TASKS)
def test_pd_torques_match_reference(task, oracle_lib):
    g = load(task)
    s = make_spec(task)
    N = g["in_actions"].shape[0]
    act = np.clip(g["in_actions"], -100, 100).astype(np.float32)
    tau = np.zeros_like(act)
    p = lambda a: a.ctypes.data  # noqa: E731
    oracle_lib.orc_compute_torques(C.byref(s.task), N, s.num_dof, p(act), p(np.ascontiguousarray(g["in_dof"])),
                                   p(g["in_last_dof_vel"]), C.c_float(s.sim_params.dt), p(tau))
    np.testing.assert_allclose(tau, g["out_torques"], **TOL)


@pytest.mark.parametrize("task", TASKS)
def test_post_physics_matches_reference(task, oracle_lib):
    g = load(task)
    s = make_spec(task)
    N = g["in_actions"].shape[0]
    b = host_buffers(s, N)
    b["root"][:] = g["in_root"]
    b["dofs"][:] = g["in_dof"]
    b["cforce"][:] = g["in_cforce"].reshape(-1, 3)
    b["rbs"][:] = g["in_rbs"].reshape(-1, 13)
    b["actions"][:] = np.clip(g["in_actions"], -100, 100)
    b["last_actions"][:] = g["in_last_actions"]
    b["last_dof_vel"][:] = g["in_last_dof_vel"]
    b["commands"][:] = g["in_commands"]
    b["feet_air_time"][:] = g["in_feet_air_time"]
    b["last_contacts"][:] = g["in_last_contacts"]
    b["episode_length"][:] = g["in_episode_length"]
    b["torques"][:] = g["in_torques"]
    E = bridge._env_struct(b)
    mh = cabi.ModelHandle(s.model)
    p = lambda a: a.ctypes.data  # noqa: E731
    oracle_lib.orc_post_physics(C.byref(mh.desc), C.byref(s.task), N, p(b["root"]), p(b["dofs"]), p(b["cforce"]),
                                p(b["rbs"]), C.byref(E), int(g["step_counter"]))
    assert g["out_reset"].sum() > 0 and g["out_time_out"].sum() > 0  # the fixture exercises resets
    np.testing.assert_array_equal(b["reset"], g["out_reset"])
    np.testing.assert_array_equal(b["time_out"], g["out_time_out"])
    np.testing.assert_array_equal(b["episode_length"], g["out_episode_length"])
    np.testing.assert_allclose(b["base_lin_vel"], g["out_base_lin_vel"], **TOL)
    np.testing.assert_allclose(b["base_ang_vel"], g["out_base_ang_vel"], **TOL)
    np.testing.assert_allclose(b["projected_gravity"], g["out_projected_gravity"], **TOL)
    np.testing.assert_allclose(b["rpy"], g["out_rpy"], **TOL)
    np.testing.assert_allclose(b["commands"], g["out_commands"], **TOL)
    np.testing.assert_allclose(b["rew"], g["out_rew"], **TOL)
    np.testing.assert_allclose(b["episode_sums"], g["out_episode_sums"], **TOL)
    np.testing.assert_allclose(b["feet_air_time"], g["out_feet_air_time"], **TOL)
    np.testing.assert_array_equal(b["last_contacts"], g["out_last_contacts"])
    np.testing.assert_allclose(b["root"], g["out_root"], **TOL)
    np.testing.assert_allclose(b["dofs"], g["out_dof"], **TOL)
    np.testing.assert_allclose(b["obs"], g["out_obs"], **TOL)
    if s.num_privileged_obs:
        np.testing.assert_allclose(b["priv_obs"], g["out_priv"], **TOL)
    np.testing.assert_allclose(b["last_actions"], g["out_last_actions"], **TOL)
    np.testing.assert_allclose(b["last_dof_vel"], g["out_last_dof_vel"], **TOL)
    # the fixture has a push step (ep_len at the push boundary, resets): last_root_vel takes
    # the reference's all-env draw of root_states[:, 7:9] (:549-550, :709) ...
    assert (g["out_root_tensor"][:, 7:9] != g["out_root"][:, 7:9]).any()
    np.testing.assert_allclose(b["last_root_vel"], g["out_last_root_vel"], **TOL)
    # ... while the state (what the simulation integrates next) keeps the envs not pushed
    # (out_root: what set_actor_root_state_tensor_indexed sent to the sim, :553-555)
    nsum = len(s.sum_names)
    means = b["episode_acc"][:nsum] / max(b["episode_acc"][nsum], 1.0) / s.max_episode_length_s
    np.testing.assert_allclose(means, g["out_extras_episode"], **TOL)
