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
