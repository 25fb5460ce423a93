"""Kernel sequence of one recurrent PPO optimizer step from a rocprofv3 kernel trace:
the kernels from the second-to-last pair of k_lstm_fwd<.., 4> launches (one step = the
actor's and the critic's memory) to the next pair.  usage: step_kernels.py <trace.csv>"""
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "k_lstm_fwd" in r[2] and ", 4>" in r[2]]
a, b = idx[-4], idx[-2]
tot = 0
for s, e, n in rows[a:b]:
    tot += e - s
    print(f"{(e - s) / 1e3:8.1f} us  {n[:120]}")
print(f"{b - a} kernels, busy {tot / 1e3:.1f} us, wall {(rows[b][0] - rows[a][0]) / 1e3:.1f} us")
