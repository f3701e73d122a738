# A/B sweep on one MI355X without the profiler: for each "NAME=value ..." setting in $SETTINGS
# (separated by ';') one bench frame at --res ${RES:-1024}; prints the value, the k-NN launch
# times and (with GI_KNN_DBG=16 in the setting) the chunk kernel's phase cycle counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ab
mkdir -p $D
i=0
IFS=';' read -ra SET <<< "$SETTINGS"
for s in "${SET[@]}"; do
  i=$((i+1))
  echo "== $s"
  env $s timeout -k 10 300 python3 bench.py --res ${RES:-1024} --steps ${STEPS:-1} --warmup ${WARMUP:-0} --no-cpu-baseline ${BENCH_ARGS:-} > $D/s$i.log 2>&1 || { tail -20 $D/s$i.log; exit 1; }
  grep '^{' $D/s$i.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['roofline']['global']; c=d['roofline']['caustic_kernel']; print('value', d['value'], 'ms', d['ms_per_step'], 'glob_ms', g['avg_launch_ms'], 'fb_ms', g['fallback_avg_ms'], 'fb_frac', g['fallback_query_frac'], 'vis', round(g['visited_per_query'],1), 'launches', g['launches'], 'caus_ms', c['avg_launch_ms'], 'caus_fb', c['fallback_query_frac'], 'caus_vis', round(c['visited_per_query'],1))"
  grep "phase cycles" $D/s$i.log | tail -1 || true
done
