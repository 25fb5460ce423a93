"""Per-kernel memory-path counters from rocprofv3 --pmc passes (tools/gpu_update_mem_pmc.sh):
the mean per dispatch of every counter of every pass, per kernel, plus derived figures
(L2 read latency, VMEM latency, L2 hit rate).  usage: pmc_mem_kernels.py <pass_dir>... """
import collections
import csv
import glob
import os
import statistics
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, cs in acc.items():
    m = {c: statistics.mean(v) for c, v in cs.items()}
    rows.append((m.get("SQ_WAVE_CYCLES", 0), k, m))
for _, k, m in sorted(rows, reverse=True)[:14]:
    print(k[:100])
    der = []
    if m.get("TCP_TCC_READ_REQ"):
        der.append(f"L2 read latency {m.get('TCP_TCC_READ_REQ_LATENCY', 0) / m['TCP_TCC_READ_REQ']:.0f} cyc")
    if m.get("SQ_INSTS_VMEM"):
        der.append(f"VMEM in flight per inst {m.get('SQ_INST_LEVEL_VMEM', 0) / m['SQ_INSTS_VMEM']:.0f} cyc")
    if m.get("TCC_HIT", 0) + m.get("TCC_MISS", 0):
        der.append(f"L2 hit {m['TCC_HIT'] / (m['TCC_HIT'] + m['TCC_MISS']):.2f}")
    print("   " + ", ".join(der))
    print("   " + "  ".join(f"{c}={v:.3g}" for c, v in sorted(m.items())))
