"""Top kernels of a rocprofv3 --stats run: usage kernel_stats_top.py <dir> [n]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} us  "
          f"{r['Name'][:110]}")
print(f"total {tot / 1e6:.2f} ms")
