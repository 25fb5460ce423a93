"""Data-parallel training through the drop-in entry point.

``python -m torch.distributed.run --nproc-per-node 2 train.py --task go2 ...``: the
unmodified ``train.py`` (run through ``tests/dp_train_wrapper.py``, which only records
each rank's result) trains on two ranks.  The box has one GPU, so both ranks bind to
``cuda:0`` and the process group falls back to gloo (RCCL refuses two ranks on one
device); on an 8-GPU node the same code binds rank r to ``cuda:r`` over RCCL.  Checked:
the ranks end with bitwise-identical parameters (one gradient all-reduce per optimizer
step, parameters broadcast from rank 0), they simulated different envs (seed + rank),
and only rank 0 wrote a run directory and checkpoints."""
import glob
import os
import shutil
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

from conftest import ROOT  # noqa: E402

PKG = os.path.join(ROOT, "unitree-rl-gym_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torchrun_train_py_two_ranks_share_one_policy(tmp_path):
    from legged_gym import LEGGED_GYM_ROOT_DIR
    exp = "pytest_dp_go2"
    logs = os.path.join(LEGGED_GYM_ROOT_DIR, "logs", exp)
    shutil.rmtree(logs, ignore_errors=True)
    env = dict(os.environ, DP_TEST_OUT=str(tmp_path), HSA_ENABLE_IPC_MODE_LEGACY="0")
    env["PYTHONPATH"] = PKG + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("LEGGED_GYM_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dp_train_wrapper.py"),
           "--task", "go2", "--num_envs", "512", "--max_iterations", "2", "--headless",
           "--experiment_name", exp, "--run_name", "dp"]
    r = subprocess.run(cmd, cwd=PKG, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, f"torchrun train.py failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    assert "data-parallel training: 2 ranks, backend gloo" in r.stdout
    res = [torch.load(tmp_path / f"rank{k}.pt", weights_only=True) for k in range(2)]
    assert [x["rank"] for x in res] == [0, 1] and all(x["world"] == 2 for x in res)
    n_dev = torch.cuda.device_count()
    for k, x in enumerate(res):  # rank -> cuda:LOCAL_RANK modulo the visible devices
        assert x["device"] == x["env_device"] == f"cuda:{k % n_dev}"
    # one policy: bitwise-identical parameters after 2 PPO iterations of 20 optimizer steps
    assert res[0]["params"].keys() == res[1]["params"].keys()
    for name, p in res[0]["params"].items():
        assert torch.equal(p, res[1]["params"][name]), name
    # ... trained on different data: each rank's envs are its own (seed + rank)
    assert not torch.equal(res[0]["obs"], res[1]["obs"])
    # logging and checkpoints on rank 0 only
    assert res[0]["log_dir"] is not None and res[1]["log_dir"] is None
    runs = glob.glob(os.path.join(logs, "*_dp"))
    assert len(runs) == 1, runs
    assert sorted(f for f in os.listdir(runs[0]) if f.endswith(".pt")) == ["model_0.pt", "model_2.pt"]
    ck = torch.load(os.path.join(runs[0], "model_2.pt"), map_location="cpu", weights_only=True)["model_state_dict"]
    for name, p in res[0]["params"].items():
        assert torch.equal(ck[name], p), name
    shutil.rmtree(logs, ignore_errors=True)
