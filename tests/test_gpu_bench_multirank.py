"""bench.py's multi-rank plumbing, executed.

``python bench.py --gpus 2`` outside a launcher starts itself under
``torch.distributed.run`` (``bench.self_launch``); each rank joins through
``legged_gym.utils.distributed.init_from_env``, the hook ``train.py`` uses.  The box
has one GPU, so both ranks bind to ``cuda:0`` and the group is gloo (RCCL refuses two
ranks on one device); on the driver's 8-GPU node the same code binds rank r to
``cuda:r`` over RCCL.  Checked: one JSON line on stdout, ``n_gpus`` 2 and ``dp2``, the
whole-job value = 2 x N x T x steps / elapsed (elapsed = the max-over-ranks timed
region, ``ms_per_step`` x steps), and a zero exit status (torchrun's: every rank)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

from conftest import ROOT  # noqa: E402


def test_bench_two_ranks_one_json_line():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("LEGGED_GYM_DIST_BACKEND", None)
    env.pop("WORLD_SIZE", None)
    steps = 2
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", "1",
           "--no_other_configs", "--no_cpu_baseline", "--env_steps", "20"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, f"bench.py --gpus 2 failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    js = [ln for ln in lines if ln.lstrip().startswith("{")]
    assert len(js) == 1 and len(lines) == 1, r.stdout
    line = json.loads(js[0])
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "dp2"
    assert line["steps"] == steps and line["warmup"] == 1
    n, t = line["config"]["num_envs_per_gpu"], 24
    elapsed = line["ms_per_step"] * 1e-3 * steps
    assert line["value"] == pytest.approx(2 * n * t * steps / elapsed, rel=1e-3)
    assert "cpu_baseline" not in line and "other_configs_env_only" not in line
