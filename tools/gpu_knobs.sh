# Knob sweep on one MI355X: for each "NAME=value ..." setting in $SETTINGS (separated by ';'),
# a kernel-trace profile of one bench frame at --res ${RES:-512}; prints the top kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/knobs
mkdir -p $D
i=0
IFS=';' read -ra SET <<< "$SETTINGS"
for s in "${SET[@]}"; do
  i=$((i+1))
  echo "== $s"
  env $s timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/s$i -o run -- python3 bench.py --res ${RES:-512} --steps 1 --warmup 0 --no-cpu-baseline > $D/s$i.log 2>&1 || { tail -20 $D/s$i.log; exit 1; }
  grep '^{' $D/s$i.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['roofline']['global']; c=d['roofline']['caustic_kernel']; print('value', d['value'], 'fb_frac', g['fallback_query_frac'], 'fb_ms', g['fallback_avg_ms'], 'glob_ms', g['avg_launch_ms'], 'caus_ms', c['avg_launch_ms'], 'caus_fb', c['fallback_query_frac'], 'caus_fb_ms', c['fallback_avg_ms'], 'caus_vis', round(c['visited_per_query'],1))"
  python3 - $D/s$i/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:9]:
    print(f'  {r["Name"][:52]:52s} {int(r["Calls"]):5d} {float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["AverageNs"])/1e6:8.3f} ms/call')
PY
done
