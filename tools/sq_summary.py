"""Instruction mix of the env-step kernel from two rocprofv3 SQ counter passes
(tools/gpu_env_profile.sh): per-launch instruction counts, per-wave counts per control step,
and the wave-time shares (quad-cycle counters over SQ_WAVE_CYCLES; MI355X_MICROARCH.md
constants table).  Written to a JSON that bench.py reads for roofline["valu"].

    python tools/sq_summary.py <pass1_counter_collection.csv> <pass2_counter_collection.csv> out.json [kernel]
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def load(path, kernel="k_step<"):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
    d = collections.defaultdict(list)
    name = None
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
    out = {k: statistics.mean(v) for k, v in d.items()}
    out["_name"] = name
    return out


def main(p1, p2, out, kernel="k_step<"):
    c = load(p1, kernel)
    c.update(load(p2, kernel))
    waves = c.get("SQ_WAVES", 4096.0)
    wc = c["SQ_WAVE_CYCLES"]
    res = {
        "kernel": c.get("_name"),
        "waves_per_launch": waves,
        "valu_insts_per_launch": c["SQ_INSTS_VALU"],
        "lds_insts_per_launch": c["SQ_INSTS_LDS"],
        "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
        "valu_insts_per_wave": c["SQ_INSTS_VALU"] / waves,
        "share_of_wave_time": {
            "issuing_valu": c["SQ_ACTIVE_INST_VALU"] / wc,
            "issuing_any": c["SQ_ACTIVE_INST_ANY"] / wc,
            "waiting_on_counters": c["SQ_WAIT_ANY"] / wc,
            "waiting_on_dependencies": c["SQ_WAIT_INST_ANY"] / wc,
        },
        "lds_bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT"),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
