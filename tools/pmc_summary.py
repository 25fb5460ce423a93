"""Summarise rocprofv3 kernel-trace / PMC csv output for one kernel into profiles/.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KiB) come from
separate passes.  Each pass also profiled a calibration copy of a known byte count
(tools/profile_env.py: 1 GiB read + 1 GiB written, float4 streaming, larger than the
Infinity Cache), so the kernel's counters are scaled by known / measured of that copy
on the same box and pass (the guide's gfx950 FETCH_SIZE x2 correction is what this
measures; a box whose counters cover only part of the channels is corrected too).
The uncorrected figures are kept beside the corrected ones.
usage: python tools/pmc_summary.py <trace_dir> <fetch_dir> <write_dir> <kernel_substr> <out.json>
"""
import csv
import glob
import json
import sys

CAL_BYTES = 1 << 30
CAL_KERNEL = "copy"  # torch's elementwise copy kernel of the calibration tensors


def rows(d, name):
    f = glob.glob(f"{d}/**/*{name}", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def counter(d, pred):
    out = []
    for r in rows(d, "counter_collection.csv"):
        if pred(r["Kernel_Name"]):
            out.append(float(r["Counter_Value"]))
    return out


def main(trace, fetch, write, kname, out):
    stats = [r for r in rows(trace, "kernel_stats.csv") if kname in r["Name"]]
    is_k = lambda n: kname in n
    is_cal = lambda n: CAL_KERNEL in n.lower() and kname not in n
    fs, ws = counter(fetch, is_k), counter(write, is_k)
    # calibration: the largest-count copy dispatches are the 1 GiB ones
    cf, cw = sorted(counter(fetch, is_cal))[-3:], sorted(counter(write, is_cal))[-3:]
    res = {"kernel": stats[0]["Name"] if stats else kname}
    if stats:
        res.update(calls=int(stats[0]["Calls"]), avg_ns=float(stats[0]["AverageNs"]), min_ns=float(stats[0]["MinNs"]),
                   max_ns=float(stats[0]["MaxNs"]))
    if fs and ws:
        f_kib, w_kib = sum(fs) / len(fs), sum(ws) / len(ws)
        res.update(fetch_size_kib=f_kib, write_size_kib=w_kib,
                   hbm_bytes_per_launch_uncorrected=(f_kib + w_kib) * 1024.0,
                   hbm_bytes_per_launch_guide_x2=(2.0 * f_kib + w_kib) * 1024.0)
        if cf and cw:
            rf = CAL_BYTES / (sum(cf) / len(cf) * 1024.0)
            rw = CAL_BYTES / (sum(cw) / len(cw) * 1024.0)
            res.update(calibration={"known_read_bytes": CAL_BYTES, "known_write_bytes": CAL_BYTES,
                                    "fetch_size_kib": sum(cf) / len(cf), "write_size_kib": sum(cw) / len(cw),
                                    "read_scale": rf, "write_scale": rw},
                       read_bytes_per_launch=f_kib * 1024.0 * rf, write_bytes_per_launch=w_kib * 1024.0 * rw,
                       hbm_bytes_per_launch=(f_kib * rf + w_kib * rw) * 1024.0)
        else:
            res.update(hbm_bytes_per_launch=res["hbm_bytes_per_launch_guide_x2"], calibration=None)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:6])
