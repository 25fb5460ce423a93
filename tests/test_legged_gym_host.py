"""legged_gym boundary on the host: registry, CLI, config, checkpoint paths,
and the loud failure of the product path without a GPU."""
import os

import pytest
import torch

import isaacgym  # noqa: F401
from legged_gym.envs import *  # noqa: F401,F403
from legged_gym.utils import get_args, task_registry
from legged_gym.utils.helpers import class_to_dict, get_load_path, update_cfg_from_args


def test_tasks_registered():
    assert set(task_registry.task_classes) >= {"go2", "g1", "h1", "h1_2"}
    env_cfg, train_cfg = task_registry.get_cfgs("go2")
    assert env_cfg.seed == train_cfg.seed == 1


def test_unknown_task_raises_value_error():
    with pytest.raises(ValueError):
        task_registry.make_env("no_such_task", args=get_args([]))
    with pytest.raises(ValueError):
        task_registry.make_alg_runner(env=None, name=None, train_cfg=None, args=get_args([]))


def test_cli_flags_of_the_reference():
    a = get_args(["--task", "h1", "--num_envs", "128", "--headless", "--sim_device", "cuda:1", "--rl_device", "cuda:1",
                  "--seed", "7", "--max_iterations", "3", "--resume", "--load_run", "x", "--checkpoint", "5",
                  "--experiment_name", "e", "--run_name", "r"])
    assert a.task == "h1" and a.num_envs == 128 and a.headless and a.sim_device == "cuda:1" and a.sim_device_id == 1
    env_cfg, train_cfg = task_registry.get_cfgs("h1")
    import copy
    env_cfg, train_cfg = copy.deepcopy(env_cfg), copy.deepcopy(train_cfg)
    update_cfg_from_args(env_cfg, train_cfg, a)
    assert env_cfg.env.num_envs == 128 and train_cfg.seed == 7 and train_cfg.runner.max_iterations == 3
    assert train_cfg.runner.resume and train_cfg.runner.load_run == "x" and train_cfg.runner.checkpoint == 5
    assert train_cfg.runner.experiment_name == "e" and train_cfg.runner.run_name == "r"


def test_class_to_dict_is_alphabetical():
    env_cfg, train_cfg = task_registry.get_cfgs("go2")
    keys = list(class_to_dict(env_cfg.rewards.scales))
    assert keys == sorted(keys)
    d = class_to_dict(train_cfg)
    assert set(d) >= {"runner", "algorithm", "policy", "seed"}


def test_get_load_path(tmp_path):
    for run in ("Jan01_00-00-00_a", "Feb01_00-00-00_b", "exported"):
        (tmp_path / run).mkdir()
    for m in ("model_50.pt", "model_100.pt", "model_0.pt"):
        (tmp_path / "Jan01_00-00-00_a" / m).write_bytes(b"")
    p = get_load_path(str(tmp_path), load_run="Jan01_00-00-00_a")
    assert p.endswith("model_100.pt")
    assert get_load_path(str(tmp_path), load_run="Jan01_00-00-00_a", checkpoint=50).endswith("model_50.pt")
    with pytest.raises(ValueError):
        get_load_path(str(tmp_path / "missing"))


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_env_refuses_to_run_without_gpu():
    with pytest.raises(RuntimeError, match="GPU|gpu"):
        task_registry.make_env("go2", args=get_args(["--num_envs", "4"]))


def test_cpu_sim_device_is_refused_not_faked():
    with pytest.raises(RuntimeError, match="no CPU physics path|GPU"):
        task_registry.make_env("go2", args=get_args(["--num_envs", "4", "--sim_device", "cpu", "--pipeline", "cpu"]))


def test_mlp_policy_export(tmp_path):
    from legged_gym.utils.helpers import export_policy_as_jit
    from rsl_rl.modules import ActorCritic
    ac = ActorCritic(48, 48, 12, [64, 32], [64, 32])
    export_policy_as_jit(ac, str(tmp_path))
    m = torch.jit.load(str(tmp_path / "policy_1.pt"))
    x = torch.randn(3, 48)
    torch.testing.assert_close(m(x), ac.actor(x))


# --- plugin API: the reference's per-step hooks run in Python; overrides the
# native step would silently ignore are refused

def test_task_step_hooks_accepted_native_overrides_refused():
    from legged_gym.envs.base.legged_robot import LeggedRobot
    from legged_gym.envs.h1.h1_env import H1Robot

    class G1Style(H1Robot):  # the reference's G1Robot pattern (g1_env.py:10-141)
        def _get_noise_scale_vec(self, cfg):
            pass

        def _init_foot(self):
            pass

        def update_feet_state(self):
            pass

        def compute_observations(self):
            pass

        def _post_physics_step_callback(self):
            pass

    G1Style._refuse_native_step_overrides()  # accepted
    assert G1Style.python_step_hooks() == {"compute_observations", "_post_physics_step_callback"}
    for name in LeggedRobot.PYTHON_STEP_HOOKS:
        cls = type("Hook_" + name, (LeggedRobot,), {name: lambda self, *a: None})
        cls._refuse_native_step_overrides()
        assert cls.python_step_hooks() == {name}
    # what stays inside the kernel is refused, at construction, before anything touches a device
    assert set(LeggedRobot.NATIVE_STEP_METHODS) == {"_compute_torques", "_resample_commands", "_push_robots",
                                                    "compute_reward", "post_physics_step", "_reset_dofs",
                                                    "_reset_root_states"}
    for name in LeggedRobot.NATIVE_STEP_METHODS:
        cls = type("Override_" + name, (LeggedRobot,), {name: lambda self, *a: None})
        with pytest.raises(NotImplementedError, match=name):
            cls._refuse_native_step_overrides()
    Torques = type("Torques", (G1Style,), {"_compute_torques": lambda self, a: a})
    with pytest.raises(NotImplementedError, match="silently ignored"):
        Torques(cfg=None, sim_params=None, physics_engine=None, sim_device="cuda:0", headless=True)

    class WithPythonTerm(LeggedRobot):  # the reward plugin point
        def _reward_knee_height(self):
            return None
    WithPythonTerm._refuse_native_step_overrides()
    assert WithPythonTerm.python_step_hooks() == frozenset()
    for t in ("go2", "g1", "h1", "h1_2"):  # the registered tasks themselves: native, no hooks
        task_registry.get_task_class(t)._refuse_native_step_overrides()
        assert task_registry.get_task_class(t).python_step_hooks() == frozenset()


def test_python_reward_terms_refresh_every_body_row():
    """A task with Python `_reward_*` terms gets every rigid_body_states row refreshed each step
    (they may read a torso or knee row, as after the reference's refresh, h1_env.py:48-56);
    without Python terms the humanoids refresh the feet rows only."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from hostspec import make_spec
    from leggedsim.task import build_task_params
    spec = make_spec("h1")
    feet = [int(i) for i in spec.feet_indices]
    assert spec.task.body_state_mask == sum(1 << b for b in feet) and spec.task.write_body_states == 1
    spec._native_reward_names = list(spec.reward_names)
    spec._py_rewards = [("knee_height", None)]
    T = build_task_params(spec)
    assert T.body_state_mask == 0 and T.write_body_states == 1 and T.num_extra_sums == 1
    spec.rigid_body_state_bodies = "feet"  # an explicit choice wins
    assert build_task_params(spec).body_state_mask == sum(1 << b for b in feet)
    q = make_spec("go2")  # a quadruped with Python terms: body rows are written too
    q._native_reward_names, q._py_rewards = list(q.reward_names), [("x", None)]
    T = build_task_params(q)
    assert T.write_body_states == 1 and T.body_state_mask == 0
    spec.rigid_body_state_bodies = "torso"
    with pytest.raises(ValueError):
        build_task_params(spec)


# --- the reference scripts' import surface

def test_logger_and_terrain_are_exported():
    from legged_gym.utils import Logger, Terrain, export_policy_as_jit, get_args, task_registry  # noqa: F401
    log = Logger(0.02)
    log.log_states({"dof_pos": 0.1, "dof_vel": 0.2})
    log.log_state("dof_pos", 0.3)
    assert log.state_log["dof_pos"] == [0.1, 0.3]
    log.log_rewards({"rew_tracking": torch.tensor(2.0), "other": torch.tensor(9.0)}, 3)
    log.log_rewards({"rew_tracking": torch.tensor(1.0)}, 1)
    assert log.rew_log["rew_tracking"] == [6.0, 1.0] and "other" not in log.rew_log and log.num_episodes == 4
    log.print_rewards()
    log.reset()
    assert not log.state_log and not log.rew_log
