#!/bin/bash
# ind_kernel cost split on C2: kernel-trace runs with GI_DBG unset / 1 (no trace or shade) /
# 2 (no sampling either); prints the kernel averages (timing only: GI_DBG changes the image).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dbgs
for v in 0 1 2; do
  if [ $v = 0 ]; then unset GI_DBG; else export GI_DBG=$v; fi
  D=gpurun_out/dbgs/d$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python3 - $D $v <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
out = []
for p in ("ind_kernel", "ind_cont", "reduce_prim", "slot0"):
    m = [r for r in rows if p in r["Name"]]
    n = sum(int(r["Calls"]) for r in m); t = sum(float(r["TotalDurationNs"]) for r in m)
    out.append(f"{p} {t / max(n, 1) / 1e6:.3f} x{n}")
print("GI_DBG=" + sys.argv[2] + ": " + " | ".join(out))
PY
done
