"""Linear fit of the k_step traffic counters against the env count (tools/gpu_traffic_sweep.sh).

Per build (shipped, I/O-only) and counter (FETCH_SIZE, WRITE_SIZE): counted bytes per launch =
intercept + slope * envs, least squares over 512 / 1024 / 2048 / 4096 envs.  The intercept is
per-launch traffic that does not scale with envs (instruction fetch, the model blob, the
parameter structs); the slope is per-env traffic.  The I/O-only build moves a known byte count
per env (tools/traffic_calib.py go2_io_bytes), so its slopes are the counters' tally factors
for this access pattern; the shipped slopes divided by them are the shipped kernel's HBM
bytes per env, compared with its own I/O bytes (<= 1.15x).  For the other
robots (no hand-counted I/O list) the comparison is tally-free: the shipped slope over the
I/O-only slope, per counter (the same access pattern, so the tally factor cancels).
usage: python tools/traffic_sweep_fit.py <sweep_dir> [out.json] [task]"""
import glob
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic_calib import go2_io_bytes  # noqa: E402


def fit(ns, ys):
    A = np.stack([np.ones(len(ns)), np.asarray(ns, float)], 1)
    (a, b), res, *_ = np.linalg.lstsq(A, np.asarray(ys, float), rcond=None)
    pred = A @ np.array([a, b])
    r2 = 1.0 - float(((np.asarray(ys) - pred) ** 2).sum()) / max(float(((np.asarray(ys) - np.mean(ys)) ** 2).sum()), 1e-30)
    return float(a), float(b), r2


def main(d, out=None, task="go2"):
    data = {}
    for f in glob.glob(os.path.join(d, "*_*", "pmc_k_step.json")):
        lib, n = os.path.basename(os.path.dirname(f)).rsplit("_", 1)
        j = json.load(open(f))
        data.setdefault(lib, []).append((int(n), j["fetch_size_kib"] * 1024.0, j["write_size_kib"] * 1024.0,
                                         j.get("avg_ns")))
    res = {"task": task}
    if task == "go2":
        rd, wr = go2_io_bytes()
        known_r, known_w = sum(rd.values()), sum(wr.values())
        res["known_io_bytes_per_env"] = {"read": known_r, "write": known_w}
    for lib, rows in data.items():
        rows.sort()
        ns = [r[0] for r in rows]
        fr, fw = fit(ns, [r[1] for r in rows]), fit(ns, [r[2] for r in rows])
        res[lib] = {"envs": ns, "fetch_bytes": [r[1] for r in rows], "write_bytes": [r[2] for r in rows],
                    "avg_ns": [r[3] for r in rows],
                    "fetch_fit": {"intercept": fr[0], "slope_per_env": fr[1], "r2": fr[2]},
                    "write_fit": {"intercept": fw[0], "slope_per_env": fw[1], "r2": fw[2]}}
    if "io" in res and "shipped" in res:
        res["shipped_over_io_per_env"] = {
            k: res["shipped"][f"{k}_fit"]["slope_per_env"] / res["io"][f"{k}_fit"]["slope_per_env"]
            for k in ("fetch", "write")}
    if "io" in res and "shipped" in res and task == "go2":
        tr = res["io"]["fetch_fit"]["slope_per_env"] / known_r  # counted bytes per true byte
        tw = res["io"]["write_fit"]["slope_per_env"] / known_w
        sr = res["shipped"]["fetch_fit"]["slope_per_env"] / tr
        sw = res["shipped"]["write_fit"]["slope_per_env"] / tw
        res["calibrated"] = {
            "read_tally": tr, "write_tally": tw,
            "shipped_read_bytes_per_env": sr, "shipped_write_bytes_per_env": sw,
            "shipped_bytes_per_env": sr + sw, "own_io_bytes_per_env": known_r + known_w,
            "ratio_to_own_io": (sr + sw) / (known_r + known_w),
            "shipped_intercept_read_bytes": res["shipped"]["fetch_fit"]["intercept"] / tr,
            "shipped_intercept_write_bytes": res["shipped"]["write_fit"]["intercept"] / tw,
            "io_intercept_read_bytes": res["io"]["fetch_fit"]["intercept"] / tr,
            "io_intercept_write_bytes": res["io"]["write_fit"]["intercept"] / tw,
        }
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt)


if __name__ == "__main__":
    main(*sys.argv[1:4])
