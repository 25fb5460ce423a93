"""A control step's extras left to the step's consumer (the captured rollout's
env step without its own extras launch).

LeggedRobot.step with `defer_extras` issues lgs_step_deferred; the rollout's next policy launch
(pmlp_rollout_forward's deferred store, or pmlp_store_step_env for the recurrent policies) does
k_step_extras' work on its own rows and once: the carried time-outs, the episode means, the
all-env push bookkeeping, the accumulator slots, the push flags and the step counter
(legged_robot.py:540-555, 742-768).  Each test checks the deferred form against lgs_step's own
extras launch, bit for bit."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402

N = 64
EXTRAS = ["_time_outs", "last_root_vel", "_d_step_counter", "root_states", "dof_state", "rew_buf", "_episode_sums"]
# sums over the reset envs by float atomics: their order is not fixed (1e-6)
ATOMIC = ["_ep_means", "_episode_acc"]


def _env(name, task="go2", push_s=None):
    env_cfg, train_cfg = task_registry.get_cfgs(task)
    env_cfg, train_cfg = copy.deepcopy(env_cfg), copy.deepcopy(train_cfg)
    if push_s is not None:
        env_cfg.domain_rand.push_robots = True
        env_cfg.domain_rand.push_interval_s = push_s
    task_registry.register(name, task_registry.get_task_class(task), env_cfg, train_cfg)
    args = get_args(["--task", name, "--num_envs", str(N), "--headless"])
    env, _ = task_registry.make_env(name=name, args=args)
    return env, args


def _same(a, b, keys=EXTRAS, atomic=ATOMIC):
    for k in keys:
        x, y = getattr(a, k), getattr(b, k)
        assert torch.equal(x, y), k
    for k in atomic:
        torch.testing.assert_close(getattr(a, k), getattr(b, k), rtol=1e-6, atol=1e-6, msg=k)


def test_deferred_step_then_extras_is_lgs_step_bitwise():
    """step(defer) + flush_extras() == step() on every buffer, through resets, a mass time-out,
    steps where some env is pushed and steps where none is (the vsim restore)."""
    a, _ = _env("go2_extras_eager", push_s=0.1)  # a push every 5 control steps
    b, _ = _env("go2_extras_defer", push_s=0.1)
    for e in (a, b):
        e.reset()
    b.defer_extras = True
    g = torch.Generator(device="cuda").manual_seed(5)
    resets = 0
    for t in range(40):
        if t == 20:
            for e in (a, b):
                e.episode_length_buf = torch.full_like(e.episode_length_buf, int(e.max_episode_length))
        act = 0.8 * torch.randn(N, a.num_actions, device="cuda", generator=g)
        oa = a.step(act)
        ob = b.step(act)
        assert "_deferred_extras" in ob[4] and "_deferred_extras" not in oa[4]
        b.flush_extras()
        resets += int(oa[3].sum())
        assert torch.equal(oa[0], ob[0]) and torch.equal(oa[3], ob[3])
        _same(a, b)
        for k in oa[4]["episode"]:
            torch.testing.assert_close(oa[4]["episode"][k], ob[4]["episode"][k], rtol=1e-6, atol=1e-6, msg=k)
    assert resets >= N  # the mass time-out (and any falls)


@pytest.mark.parametrize("task", ["go2", "h1"])
def test_rollout_consumes_the_deferred_extras_bitwise(task):
    """OnPolicyRunner with the env's extras in the rollout's launches (the default) == the env's
    own extras launch (runner cfg defer_env_extras = False): parameters, rollout storage and
    every extras buffer after three iterations (eager, captured, replayed)."""
    runs = []
    for defer in (True, False):
        env_cfg, train_cfg = task_registry.get_cfgs(task)
        env_cfg, train_cfg = copy.deepcopy(env_cfg), copy.deepcopy(train_cfg)
        train_cfg.runner.defer_env_extras = defer
        name = f"{task}_defer_{int(defer)}"
        task_registry.register(name, task_registry.get_task_class(task), env_cfg, train_cfg)
        args = get_args(["--task", name, "--num_envs", str(N), "--headless"])
        env, _ = task_registry.make_env(name=name, args=args)
        runner, _ = task_registry.make_alg_runner(env=env, name=name, args=args, log_root=None)
        runner.learn(3)
        torch.cuda.synchronize()
        assert runner._rollout_graph is not None
        assert not env.defer_extras  # off outside the collection loop
        runs.append((env, runner))
    (ea, ra), (eb, rb) = runs
    for pa, pb in zip(ra.alg.actor_critic.parameters(), rb.alg.actor_critic.parameters()):
        assert torch.equal(pa, pb)
    for k in ("observations", "rewards", "actions", "values", "dones", "actions_log_prob"):
        assert torch.equal(getattr(ra.alg.storage, k), getattr(rb.alg.storage, k)), k
    # (the deferred consumer zeroes the next step's accumulator slot, not the one it read)
    _same(ea, eb, atomic=["_ep_means"])
    for e in (ea, eb):
        assert not e._episode_acc[e._buf_idx ^ 1].any()  # the slot the next step adds into
    assert ea.common_step_counter == eb.common_step_counter
