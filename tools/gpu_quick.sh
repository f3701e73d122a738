# Iteration loop on one MI355X: GPU parity tests, the C2 bench line (no CPU baseline) and a
# kernel-trace profile of one C2 frame. Extra env (GI_* knobs) passes through.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/quick
mkdir -p $D
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 ${TESTS:-} > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
  tail -2 $D/pytest_gpu.log
fi
timeout -k 10 600 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-900
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/quick/trace/run_kernel_stats.csv")))
for r in rows[:14]:
    print(f'{r["Name"][:58]:58s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e6:10.1f} ms {float(r["AverageNs"])/1e6:8.3f} ms/call')
PY
