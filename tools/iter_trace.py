"""Break down the last PPO iteration in a rocprofv3 kernel trace (csv or csv.gz):
wall span, busy time, idle gaps, and the top kernels of the collection and update
phases.  usage: iter_trace.py <run_kernel_trace.csv[.gz]> [steps_per_env=24]"""
import collections
import csv
import gzip
import sys

path = sys.argv[1]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 24
f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(f)]
rows.sort()
steps = [i for i, r in enumerate(rows) if r[2].startswith("void k_step")]
# last iteration = the last T k_step launches; the previous iteration's last k_step bounds it
first = steps[-T]
prev_end = max(i for i in range(first) if rows[i][2].startswith("void k_step")) if len(steps) > T else 0
# the iteration starts after the previous k_step's update: take the first kernel after the previous
# iteration's update, approximated as the first of the T act kernels before k_step #first
start = first
adam = [i for i in range(prev_end, first) if rows[i][2].startswith("k_adam")]
if adam:  # the collection starts right after the previous update's last optimizer step
    start = adam[-1] + 1
else:
    while start > prev_end + 1 and not rows[start - 1][2].startswith("void k_step") and \
            rows[first][0] - rows[start - 1][0] < 2e6:
        start -= 1
upd0 = steps[-1] + 1
end = len(rows)


def phase(lo, hi, name):
    seg = rows[lo:hi]
    if not seg:
        return
    wall = seg[-1][1] - seg[0][0]
    busy = sum(e - s for s, e, _ in seg)
    gaps = sum(max(0, seg[i + 1][0] - seg[i][1]) for i in range(len(seg) - 1))
    print(f"== {name}: {len(seg)} kernels, wall {wall / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle gaps {gaps / 1e6:.3f} ms")
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n in seg:
        agg[n][0] += e - s
        agg[n][1] += 1
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:18]:
        print(f"   {t / 1e3:8.1f} us  n={c:4d} avg {t / c / 1e3:6.1f}  {n[:100]}")


phase(start, upd0, "collection")
phase(upd0, end, "update (to end of trace)")
