"""Tabulate `hipcc -Rpass-analysis=kernel-resource-usage` output (VGPR/AGPR/scratch/occupancy/LDS
per kernel): python tools/resource_table.py remarks.txt [name-filter]"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read().splitlines()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows, cur = [], None
for line in txt:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for k in ("VGPRs", "AGPRs", r"ScratchSize \[bytes/lane\]", r"Occupancy \[waves/SIMD\]", r"LDS Size \[bytes/block\]"):
        m = re.search(k + r": (\d+)", line)
        if m and cur is not None:
            cur[k.split()[0]] = int(m.group(1))
rows = [r for r in rows if flt in r["name"]]
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    print(f"{d[:70]:70s} V{r.get('VGPRs')} A{r.get('AGPRs')} scratch{r.get('ScratchSize')} occ{r.get('Occupancy')} "
          f"lds{r.get('LDS')}")
