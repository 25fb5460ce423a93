"""Wave timeline of one fused-step launch (stamps build: LEGGEDSIM_LIB=.../libleggedsim_stamps.so).

Every wave records shader-clock and 100 MHz real-time stamps at kernel entry and exit and the
SIMD / CU / SE / XCC it ran on (leggedsim.hip STAMP_BEGIN / STAMP_END).  Reported for the last
of 30 control steps: the launch's span, the waves' durations, how late the last wave started,
the shader clock, how many waves shared each SIMD, and how much of the span the slowest SIMD
and the tail after the median wave's end take.
usage: LEGGEDSIM_LIB=... python tools/wave_timeline.py [task] [n] [actions_scale]"""
import ctypes as C
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from leggedsim import native  # noqa: E402


def main(task="go2", n=4096, scale=0.5):
    env, _ = task_registry.make_env(name=task, args=get_args(["--task", task, "--num_envs", str(n), "--headless"]))
    lib = native.load()
    buf = torch.zeros(n, 24, dtype=torch.int64, device="cuda")
    lib.lgs_debug_set_phase_buffer.argtypes = [C.c_void_p]
    native.check(lib, lib.lgs_debug_set_phase_buffer(buf.data_ptr()), "set_phase_buffer")
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(30):
        env.step(scale * torch.randn(n, env.num_actions, device="cuda", generator=g))
    torch.cuda.synchronize()
    b = buf.cpu().numpy().astype(np.int64)
    reset = env.reset_buf.cpu().numpy().astype(bool)
    envs = np.nonzero(b[:, 19] > 0)[0]
    b = b[envs]  # the rows lane 0 of a wave wrote (its first env)
    t0, t1, r0, r1 = b[:, 18], b[:, 19], b[:, 20], b[:, 21]
    hw, xcc = b[:, 22].astype(np.uint32), b[:, 23].astype(np.uint32)
    clk = np.median((t1 - t0) / np.maximum(r1 - r0, 1)) * 100.0  # MHz
    us = lambda ticks: ticks / 100.0  # noqa: E731  (real-time ticks at 100 MHz)
    R0 = r0.min()
    span = us(r1.max() - R0)
    dur = us(r1 - r0)
    start = us(r0 - R0)
    print(f"{task} n={n} actions x{scale}: {len(b)} waves, launch span {span:.1f} us, shader clock {clk:.0f} MHz")
    print(f"  wave duration us: min {dur.min():.1f} p10 {np.percentile(dur, 10):.1f} median {np.median(dur):.1f} "
          f"p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f}")
    print(f"  wave start us after the first: p50 {np.median(start):.2f} p99 {np.percentile(start, 99):.2f} "
          f"max {start.max():.2f}")
    print("  waves started by (us): " + ", ".join(f"{q:.0f}: {int((start <= q).sum())}" for q in
                                                 (1, 10, 50, 100, 150, 200, 250, 300, 400)))
    simd = collections.Counter()
    per_simd_end = collections.defaultdict(float)
    for k in range(len(b)):
        key = (int(xcc[k]) & 0xF, (int(hw[k]) >> 13) & 7, (int(hw[k]) >> 12) & 1, (int(hw[k]) >> 8) & 15,
               (int(hw[k]) >> 4) & 3)
        simd[key] += 1
        per_simd_end[key] = max(per_simd_end[key], us(r1[k] - R0))
    hist = collections.Counter(simd.values())
    print(f"  SIMDs used {len(simd)}; waves per SIMD histogram {dict(sorted(hist.items()))}; "
          f"CUs used {len({k[:4] for k in simd})}; XCCs {sorted({k[0] for k in simd})}")
    for c in sorted(hist):
        ends = [per_simd_end[k] for k, v in simd.items() if v == c]
        print(f"    SIMDs with {c} waves: last wave ends at median {np.median(ends):.1f} us, max {max(ends):.1f} us")
    ends = np.sort(us(r1 - R0))
    half = ends[len(ends) // 2]
    names = ["fk", "inertia", "bias_rnea", "composite", "M+rhs", "chol", "qdd", "contact_det", "rows_J", "Y",
             "A", "pgs", "z+back", "integ", "bodies", "post", "store"]
    order = np.argsort(dur)
    med = np.median(b[:, 1:18], 0)
    epw = 2 if len(b) * 2 == n else 1
    r_wave = reset[envs] | (reset[np.minimum(envs + 1, n - 1)] if epw == 2 else False)
    print(f"  waves with a reset env: {int(r_wave.sum())}, their median duration {np.median(dur[r_wave]) if r_wave.any() else 0:.1f} us "
          f"vs {np.median(dur[~r_wave]):.1f} us without")
    print("  slowest waves (phase cycles minus the median wave's, top 3 phases):")
    for k in order[::-1][:8]:
        d = b[k, 1:18] - med
        top = np.argsort(d)[::-1][:3]
        print(f"    env {envs[k]:5d} {dur[k]:6.1f} us reset {bool(r_wave[k])}: " +
              ", ".join(f"{names[i]} +{d[i]:.0f}" for i in top))
    print(f"  half the waves done at {half:.1f} us, 90 % at {ends[int(0.9 * len(ends))]:.1f} us, "
          f"all at {ends[-1]:.1f} us (tail after the median end: {100 * (ends[-1] - half) / span:.0f} % of the span)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "go2", int(sys.argv[2]) if len(sys.argv) > 2 else 4096,
         float(sys.argv[3]) if len(sys.argv) > 3 else 0.5)
