#!/bin/bash
# Kernel-trace profile of one bench.py configuration: NAME=<dir> tools/gpu_prof_args.sh <bench args>
# -> gpurun_out/prof_<NAME>/ (kernel stats csv + the bench line); prints the top kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/prof_${NAME:-x}
mkdir -p $D
timeout -k 10 ${TLIM:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py "$@" --no-cpu-baseline > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | tail -1 | cut -c1-600
f=$(find $D -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% n={r["Calls"]:>6} {r["Name"][:110]}')
print(f"total {tot/1e6:.1f} ms")
PY
