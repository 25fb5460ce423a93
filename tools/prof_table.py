"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (usage: prof_table.py <csv> [n] [divisor])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
div = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot / 1e6:.3f} ms  (per unit {tot / 1e6 / div:.3f} ms)")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / div:8.3f} ms/unit n={int(r['Calls']) / div:6.1f} "
          f"avg {float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:95]}")
