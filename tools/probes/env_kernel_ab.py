"""A/B of the fused env step across builds of libleggedsim (LEGGEDSIM_LIB): back-to-back
lgs_step launches between HIP events (bench.env_kernel_rate), alternating the builds over
several rounds in fresh processes so clock drift hits both arms alike.

usage: python tools/probes/env_kernel_ab.py LIB_A LIB_B [task:envs ...] [--rounds R]
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
out = {{}}
for task, n in {cfgs!r}:
    out[f"{{task}}:{{n}}"] = bench.env_kernel_rate(task, n, "cuda:0", 100, get_args, task_registry)["env_step_kernel_ms"]
print("RESULT", json.dumps(out), flush=True)
"""


def main():
    args = sys.argv[1:]
    rounds = 3
    if "--rounds" in args:
        i = args.index("--rounds")
        rounds = int(args[i + 1])
        del args[i:i + 2]
    libs, cfgs = args[:2], [(c.split(":")[0], int(c.split(":")[1])) for c in args[2:]] or [("go2", 4096)]
    code = CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "unitree-rl-gym_amd"), cfgs=cfgs)
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            p = subprocess.run([sys.executable, "-c", code], env={**os.environ, "LEGGEDSIM_LIB": lib},
                               capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(lib, "FAILED", p.returncode, p.stderr[-2000:], flush=True)
                sys.exit(1)
            res[lib].append(json.loads(line[0][7:]))
            print(r, os.path.basename(lib), res[lib][-1], flush=True)
    for lib in libs:
        best = {k: min(x[k] for x in res[lib]) for k in res[lib][0]}
        print("best", os.path.basename(lib), best, flush=True)


if __name__ == "__main__":
    main()
