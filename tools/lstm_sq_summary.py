"""SQ instruction mix / wave-time shares of the LSTM and heads kernels in a recurrent PPO run,
per (kernel, grid size) -- the rollout's single steps and the update's sequences apart.
usage: python tools/lstm_sq_summary.py <pass1 dir> <pass2 dir> out.json"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("k_lstm_fwd_mfma8", "k_lstm_bwd_mfma", "k_heads_fwd", "k_heads_bwd")


def load(path):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = next((k for k in KERNELS if k in name), None)
        if k is None:
            continue
        key = f"{k} grid={r['Grid_Size']} wg={r['Workgroup_Size']} vgpr={r.get('VGPR_Count', '?')}"
        d[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in d.items()}


a, b = load(sys.argv[1]), load(sys.argv[2])
out = {}
for k in sorted(set(a) | set(b)):
    c = dict(a.get(k, {}))
    c.update(b.get(k, {}))
    wc = c.get("SQ_WAVE_CYCLES")
    waves = c.get("SQ_WAVES")
    if not wc or not waves:
        continue
    out[k] = {
        "waves": waves,
        "valu_per_wave": c["SQ_INSTS_VALU"] / waves,
        "lds_per_wave": c["SQ_INSTS_LDS"] / waves,
        "salu_per_wave": c.get("SQ_INSTS_SALU", 0) / waves,
        "wave_cycles_per_wave": wc / waves,
        "issuing_valu": c["SQ_ACTIVE_INST_VALU"] / wc,
        "issuing_any": c["SQ_ACTIVE_INST_ANY"] / wc,
        "waiting_on_counters": c["SQ_WAIT_ANY"] / wc,
        "waiting_on_dependencies": c["SQ_WAIT_INST_ANY"] / wc,
        "lds_bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT"),
    }
json.dump(out, open(sys.argv[3], "w"), indent=1)
for k, v in out.items():
    print(k)
    print("   ", {kk: round(vv, 3) if isinstance(vv, float) else vv for kk, vv in v.items()})
