"""A/B of the recurrent PPO iteration (H1 / H1_2 / G1, LSTM 64): LSTM_MFMA=0 (fp32 VALU
sequence kernels and the autograd update) against the default matrix-core kernels with the
fused recurrent step.
Each variant runs in its own process (the switches are read once per process).

usage: python tools/probes/recurrent_iter_ab.py [task] [num_envs] [iters]
       python tools/probes/recurrent_iter_ab.py --inproc [task] [num_envs] [iters]
         (one run in this process with the caller's environment, for rocprofv3)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r"""
import json, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {pkg!r})
import bench
import isaacgym  # noqa: F401
from legged_gym.envs import task_registry
from legged_gym.utils import get_args
print("RESULT", json.dumps(bench.ppo_iter_rate({task!r}, {n}, "cuda:0", {iters}, 2, get_args, task_registry)), flush=True)
"""


def main():
    if sys.argv[1:2] == ["--inproc"]:
        del sys.argv[1]
        task = sys.argv[1] if len(sys.argv) > 1 else "h1"
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
        iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
        exec(CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "unitree-rl-gym_amd"), task=task, n=n, iters=iters))
        return
    task = sys.argv[1] if len(sys.argv) > 1 else "h1"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    code = CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "unitree-rl-gym_amd"), task=task, n=n, iters=iters)
    for name, env in (("fp32", {"LSTM_MFMA": "0"}), ("mfma_split_bf16", {"LSTM_MFMA": "1"})):
        r = subprocess.run([sys.executable, "-c", code], env={**os.environ, **env}, capture_output=True, text=True,
                           timeout=300)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(name, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
            sys.exit(1)
        res = json.loads(line[0][7:])
        print(name, task, n, "ppo_iter_ms", res["ppo_iter_ms"], "env_steps_per_s", res["env_steps_per_s"], flush=True)


if __name__ == "__main__":
    main()
