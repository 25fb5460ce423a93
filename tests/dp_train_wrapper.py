"""Runs the build's ``legged_gym/scripts/train.py`` unmodified (``runpy``, as ``__main__``,
with the command line it was given) under ``torch.distributed.run``, and records what
each rank ended with for ``tests/test_gpu_dp_train.py``: the rank's device, world size,
log directory and final policy parameters.  Test infrastructure only: the one thing it
adds is a wrapper around ``OnPolicyRunner.learn`` that saves those after training."""
import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "unitree-rl-gym_amd")
sys.path.insert(0, PKG)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402

OUT = os.environ["DP_TEST_OUT"]
_learn = OnPolicyRunner.learn


def learn(self, *a, **k):
    r = _learn(self, *a, **k)
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.save({"rank": rank, "world": dist.get_world_size() if dist.is_initialized() else 1,
                "backend": dist.get_backend() if dist.is_initialized() else None,
                "device": str(self.device), "env_device": str(self.env.device), "log_dir": self.log_dir,
                "obs": self.env.get_observations().detach().cpu(),
                "params": {n: p.detach().cpu() for n, p in self.alg.actor_critic.state_dict().items()}},
               os.path.join(OUT, f"rank{rank}.pt"))
    return r


OnPolicyRunner.learn = learn
script = os.path.join(PKG, "legged_gym", "scripts", "train.py")
sys.argv = [script] + sys.argv[1:]
runpy.run_path(script, run_name="__main__")
