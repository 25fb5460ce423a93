"""Per-dispatch table of one captured fused optimizer step (Go2 update) from rocprofv3 output:
duration (kernel trace) and FETCH_SIZE / WRITE_SIZE (separate counter passes) of the 7
launches after the last k_mlp_fwd<96 dispatch, in launch order -- the two 128 x 128 backward
pairs share a kernel name, so the per-name averages of pmc_summary.py mix them.
usage: python tools/probes/update_dispatches.py <trace_dir> <fetch_dir> <write_dir>"""
import csv
import glob
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)[0]
    return list(csv.DictReader(open(f)))


def last_step(seq, key):
    idx = [i for i, r in enumerate(seq) if "k_mlp_fwd<96" in key(r)]
    i = idx[-2]  # the second-to-last step: whole
    return seq[i:i + 7]


def main(tr, fe, wr):
    t = sorted(rows(tr, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    steps = last_step(t, lambda r: r["Kernel_Name"])

    def pmc(d, name):
        acc = {}
        for r in rows(d, "*counter_collection.csv"):
            if r["Counter_Name"] == name:
                acc[int(r["Dispatch_Id"])] = (r["Kernel_Name"], float(r["Counter_Value"]))
        seq = [acc[k] for k in sorted(acc)]
        return last_step(seq, lambda r: r[0])

    f, w = pmc(fe, "FETCH_SIZE"), pmc(wr, "WRITE_SIZE")
    print(f"{'kernel':70s} {'us':>7s} {'FETCH MB':>9s} {'WRITE MB':>9s}")
    for r, a, b in zip(steps, f, w):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print(f"{r['Kernel_Name'][:70]:70s} {us:7.1f} {a[1] / 1024:9.2f} {b[1] / 1024:9.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
