# Instruction-cache counters of the fused env step (k_step is ~100 KB of code per shape):
# SQC_ICACHE_* (per SQ) in one pass, the wave's instruction-fetch counters in another.
# usage: bash tools/gpu_icache.sh [task:envs ...]   (default go2:4096 h1:8192)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFGS="${@:-go2:4096 h1:8192}"
for cfg in $CFGS; do
  task=${cfg%%:*}; n=${cfg##*:}
  O=gpurun_out/icache/${task}_$n
  rm -rf $O && mkdir -p $O
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d $O/ic -o run --output-format csv -- python tools/profile_env.py $task $n 8 > $O/ic.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_BUSY_CYCLES -d $O/if -o run --output-format csv -- python tools/profile_env.py $task $n 8 > $O/if.log 2>&1 || exit 3
  python - $O <<'EOF' > $O/summary.txt || exit 4
import collections, csv, glob, statistics, sys
o = sys.argv[1]
d = collections.defaultdict(list)
for p in ("ic", "if"):
    f = glob.glob(f"{o}/{p}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "k_step<" in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {k: statistics.mean(v) for k, v in d.items()}
for k in sorted(c):
    print(f"{k:32s} {c[k]:16.1f}")
req = c.get("SQC_ICACHE_REQ") or 1.0
print(f"icache hit rate {c.get('SQC_ICACHE_HITS', 0) / req:.4f}  miss rate {c.get('SQC_ICACHE_MISSES', 0) / req:.4f}  dup-miss share {c.get('SQC_ICACHE_MISSES_DUPLICATE', 0) / req:.4f}")
print(f"wait_inst_any / wave_cycles {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.4f}")
print(f"ifetch per wave {c['SQ_IFETCH'] / c['SQ_WAVES']:.1f}  ifetch_level/ifetch (avg fetch latency, cycles) {c['SQ_IFETCH_LEVEL'] / max(c['SQ_IFETCH'], 1):.1f}")
EOF
  find $O -name "*counter_collection.csv" -size +2M -delete
  cat $O/summary.txt
done
