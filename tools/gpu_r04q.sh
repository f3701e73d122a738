#!/bin/bash
# Kernel-trace stats of C2 (bench --steps 1 --warmup 1) with exp/base/libgi_amd.so and the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kq
for v in base new; do
  L=""; [ $v = base ] && L=$GRAFT_REPO_ROOT/exp/base/libgi_amd.so
  GI_AMD_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kq/$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/kq/$v.log 2>&1 || { tail -5 gpurun_out/kq/$v.log; exit 1; }
done
python3 - <<'PY'
import csv
def load(v):
    return {r['Name']: float(r['TotalDurationNs']) / 1e6 for r in csv.DictReader(open(f'gpurun_out/kq/{v}/run_kernel_stats.csv'))}
b, n = load('base'), load('new')
rows = sorted(set(b) | set(n), key=lambda k: -max(b.get(k, 0), n.get(k, 0)))
for k in rows[:25]:
    print(f"{b.get(k,0):9.1f} {n.get(k,0):9.1f} {n.get(k,0)-b.get(k,0):+8.1f}  {k[:90]}")
PY
