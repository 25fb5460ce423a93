"""Per-kernel SQ summary from rocprofv3 counter passes (tools/gpu_update_pmc.sh): mean over
dispatches of each counter, per kernel name, with the wave-time shares.
usage: python tools/pmc_kernels.py <pass1_dir> <pass2_dir> <trace_dir>"""
import collections
import csv
import glob
import os
import statistics
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in d2.items()} for k, d2 in acc.items()}


def main(p1, p2, tr):
    a, b = load(p1), load(p2)
    st = {}
    f = glob.glob(os.path.join(tr, "**", "*kernel_stats.csv"), recursive=True)
    if f:
        for r in csv.DictReader(open(f[0])):
            st[r["Name"]] = float(r["AverageNs"])
    rows = []
    for k in a:
        c = dict(a[k])
        c.update(b.get(k, {}))
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        rows.append((st.get(k, 0.0), k, c, wc))
    rows.sort(key=lambda x: -x[0])
    for ns, k, c, wc in rows[:16]:
        w = c.get("SQ_WAVES", 1) or 1
        print(f"{ns / 1e3:7.1f} us  {k[:90]}")
        print(f"     waves {w:.0f}  VALU/wave {c.get('SQ_INSTS_VALU', 0) / w:.0f}  LDS/wave {c.get('SQ_INSTS_LDS', 0) / w:.0f}"
              f"  MFMA/wave {c.get('SQ_INSTS_MFMA', 0) / w:.0f}  share: valu {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f}"
              f" any {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} wait_cnt {c.get('SQ_WAIT_ANY', 0) / wc:.2f}"
              f" wait_dep {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} lds_wait {c.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}"
              f" lds_active {c.get('SQ_ACTIVE_INST_LDS', 0) / wc:.2f} bank_conf {c.get('SQ_LDS_BANK_CONFLICT', 0):.0f}"
              f" mfma_busy {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):.0f} busy {c.get('SQ_BUSY_CYCLES', 0):.0f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
