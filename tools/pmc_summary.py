"""Summarise rocprofv3 kernel-trace / PMC csv output for one kernel into profiles/.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB,
collected in separate passes; on gfx950 FETCH_SIZE reports half the bytes of a
wide coalesced stream, so it is doubled (that correction is calibrated for
16-B/lane loads; this kernel's 4-B loads are uncalibrated).
usage: python tools/pmc_summary.py <trace_dir> <fetch_dir> <write_dir> <kernel_substr> <out.json>
"""
import csv
import glob
import json
import sys


def rows(d, name):
    f = glob.glob(f"{d}/*{name}")
    return list(csv.DictReader(open(f[0]))) if f else []


def main(trace, fetch, write, kname, out):
    stats = [r for r in rows(trace, "kernel_stats.csv") if kname in r["Name"]]
    fs = [float(r["Counter_Value"]) for r in rows(fetch, "counter_collection.csv") if kname in r["Kernel_Name"]]
    ws = [float(r["Counter_Value"]) for r in rows(write, "counter_collection.csv") if kname in r["Kernel_Name"]]
    res = {"kernel": stats[0]["Name"] if stats else kname}
    if stats:
        res.update(calls=int(stats[0]["Calls"]), avg_ns=float(stats[0]["AverageNs"]), min_ns=float(stats[0]["MinNs"]),
                   max_ns=float(stats[0]["MaxNs"]))
    if fs and ws:
        f_kib, w_kib = sum(fs) / len(fs), sum(ws) / len(ws)
        res.update(fetch_size_kib=f_kib, write_size_kib=w_kib,
                   hbm_bytes_per_launch=(2.0 * f_kib + w_kib) * 1024.0,
                   hbm_bytes_per_launch_uncorrected=(f_kib + w_kib) * 1024.0)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:6])
