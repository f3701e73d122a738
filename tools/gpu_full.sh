# Round-end measurement on one MI355X: GPU parity tests, the default (C2) bench line with the
# CPU baseline, a kernel-trace profile of the same workload and a FETCH_SIZE PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out/full
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/full/pytest_gpu.log
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/full/bench.log 2>&1 || { tail -20 gpurun_out/full/bench.log; exit 1; }
tail -1 gpurun_out/full/bench.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/full/trace.log 2>&1 || { tail -20 gpurun_out/full/trace.log; exit 1; }
tail -1 gpurun_out/full/trace.log
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/full/pmc -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/full/pmc.log 2>&1 || { tail -20 gpurun_out/full/pmc.log; exit 1; }
echo ok
