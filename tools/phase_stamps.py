"""Per-phase cycle breakdown of the fused step (diagnostic build with s_memtime stamps).
usage: LEGGEDSIM_LIB=.../libleggedsim_stamps.so python tools/phase_stamps.py [task] [n]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from leggedsim import native  # noqa: E402

NAMES = {1: "fk", 2: "inertia", 3: "bias_rnea", 4: "composite", 5: "mass_matrix+rhs", 6: "cholesky",
         7: "qdd+qf", 8: "limits+contact_detect", 9: "contact_rows_J", 10: "Y=L^-1J^T", 11: "A=YtY", 12: "pgs",
         13: "z+backsub+cforce", 14: "integrate", 15: "body_states", 16: "post_physics", 17: "store"}


def main(task="go2", n=4096):
    args = get_args(["--task", task, "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name=task, args=args)
    lib = native.load()
    buf = torch.zeros(n, 24, dtype=torch.int64, device="cuda")
    lib.lgs_debug_set_phase_buffer.argtypes = [C.c_void_p]
    native.check(lib, lib.lgs_debug_set_phase_buffer(buf.data_ptr()), "set_phase_buffer")
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(30):
        env.step(0.5 * torch.randn(n, env.num_actions, device="cuda", generator=g))
    torch.cuda.synchronize()
    # lane 0 of each wave writes its row: with two envs per wave only the even envs have one
    rows = buf.double()
    rows = rows[rows[:, 1:18].sum(1) > 0]
    b = rows.mean(0).cpu().numpy()
    dec = env.cfg.control.decimation
    tot = b[1:18].sum()
    print(f"{task} n={n}: cycles per control step (lane-0 wave view, mean over {rows.shape[0]} waves), decimation {dec}: total {tot:.0f}")
    for i in range(1, 18):
        print(f"  {NAMES[i]:24s} {b[i]:10.0f}  {100 * b[i] / tot:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "go2", int(sys.argv[2]) if len(sys.argv) > 2 else 4096)
