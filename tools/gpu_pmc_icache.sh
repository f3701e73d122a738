#!/bin/bash
# Instruction-cache behaviour per kernel on a C2 (or BENCH_ARGS) frame: one SQ PMC pass
# (SQC_ICACHE_* requests / hits / misses, wave counts), printed per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmcicache${TAG:-}
mkdir -p $D
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $D/p1 -o run -- $B > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
python3 - $D/p1/run_counter_collection.csv <<'PY' | tee $D/summary.txt
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
print(f"{'kernel':60s} {'req':>12s} {'hit%':>6s} {'miss':>10s} {'missdup':>10s} {'req/wave':>9s}")
for n, v in rows[:20]:
    req = v.get("SQC_ICACHE_REQ", 0)
    print(f"{n[-60:]:60s} {req:12.0f} {100 * v.get('SQC_ICACHE_HITS', 0) / max(req, 1):6.2f} "
          f"{v.get('SQC_ICACHE_MISSES', 0):10.0f} {v.get('SQC_ICACHE_MISSES_DUPLICATE', 0):10.0f} "
          f"{req / max(v.get('SQ_WAVES', 1), 1):9.1f}")
PY
