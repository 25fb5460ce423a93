"""The captured PPO update replayed from one state gives the same parameters every time.

None of the update's kernels accumulates with atomics, so a replay that differs is a race
(the LSTM backward's weight-gradient waves once zeroed an LDS tile that other
waves were already filling, 17 divergent replays in 10,000 at H1 x 8192).  The same check as
tools/probes/update_race.py, shorter: the recurrent step (H1) and the MLP step (Go2)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402


@pytest.mark.parametrize("task,envs,replays", [("h1", 2048, 600), ("go2", 2048, 600)])
def test_update_replays_are_identical(task, envs, replays):
    args = get_args(["--task", task, "--num_envs", str(envs), "--headless"])
    env, _ = task_registry.make_env(name=task, args=args)
    r, _ = task_registry.make_alg_runner(env=env, name=task, args=args, log_root=None)
    r.learn(2)
    alg, st = r.alg, r.alg.storage
    if alg._rfused is not None:
        f, graph, extra = alg._rfused, alg._rgraph, []
    else:
        f, graph = alg._fused, alg._fgraph
        extra = [w for ws in f.wb for w in ws] + ([w for ws in f.wf for w in ws] if f.wf else [])
    assert f is not None and graph is not None
    state = [f.flat, f.exp_avg, f.exp_avg_sq, f.step_t, alg._lr, st.advantages, st.returns] + extra
    snap = [t.clone() for t in state]

    def replay():
        for t, s in zip(state, snap):
            t.copy_(s)
        graph.replay()

    replay()
    ref = f.flat.clone()
    assert not torch.equal(ref, snap[0])  # the replay did update the parameters
    bad = torch.zeros((), dtype=torch.int64, device=ref.device)
    for _ in range(replays):
        replay()
        bad += (f.flat != ref).any().to(torch.int64)
    assert int(bad) == 0, f"{int(bad)} of {replays} replays differ"
