# One kernel-trace run of the default bench (1 warmup + 1 step) under rocprofv3 into
# gpurun_out/trace_${TAG:-x}/, then tools/batch_timeline.py prints the per-batch kernel split.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/trace_${TAG:-x}
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | tail -1 | cut -c1-400
python3 tools/batch_timeline.py $D/run_kernel_trace.csv | tail -${LINES_OUT:-28}
