#!/bin/bash
# ind_kernel time split on a C2 frame: default, GI_DBG=1 (diffuse sample, no trace/shade),
# GI_DBG=2 (no sample, no trace) -- images meaningless under GI_DBG, only the kernel times count.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/indsplit
mkdir -p $D
for v in 0 1 2; do
  GI_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/t$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $D/t$v.log 2>&1 || { tail -5 $D/t$v.log; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$D/t$v/run_kernel_stats.csv')):
    if 'ind_kernel' in r['Name'] or 'ind_cont' in r['Name'] or 'primary_kernel' in r['Name']: print('dbg $v', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6,3))
"
done
