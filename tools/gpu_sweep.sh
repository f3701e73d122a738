# Render-workload sweep of one environment knob on one MI355X.
#   SWEEP="GI_KNN_DBG=0,1,2,4" RES=512 bash tools/gpu_sweep.sh
# Prints, per value, the frame rate and the per-map k-NN launch timings from bench.py's line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
name=${SWEEP%%=*}
vals=${SWEEP#*=}
for v in ${vals//,/ }; do
  env "$name=$v" timeout -k 10 600 python bench.py --res ${RES:-512} --steps ${STEPS:-1} --warmup 1 \
      --no-cpu-baseline > gpurun_out/sweep/$name-$v.log 2>&1 || { tail -20 gpurun_out/sweep/$name-$v.log; exit 1; }
  python3 - "$name=$v" gpurun_out/sweep/$name-$v.log <<'EOF'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = j["roofline"]
g, c = r["global"], r["caustic_kernel"]
print(f'{sys.argv[1]}: {j["value"]:.4f} {j["unit"]} ms/frame={j["ms_per_step"]:.1f} | global '
      f'{g["avg_launch_ms"]:.2f} ms/launch (fallback {g["fallback_avg_ms"]:.2f}, '
      f'{g["fallback_query_frac"]:.3f} of q) x{g["launches"]:.0f} vis={g["visited_per_query"]:.0f} | '
      f'caustic {c["avg_launch_ms"]:.2f} ms/launch', flush=True)
EOF
  grep "k-NN phase" gpurun_out/sweep/$name-$v.log | tail -1 || true
done
