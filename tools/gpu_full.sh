# Round-end measurement on one MI355X: GPU parity tests, the default (C2) bench line with the
# CPU baseline (after a FETCH_SIZE PMC pass whose traffic it reports), and a kernel-trace profile
# of the same workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out/full
rm -f gpurun_out/full/parity_l2.jsonl
GI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/full/parity_l2.jsonl timeout -k 10 900 python -u -m pytest ${PYTEST_TARGET:-tests} -x -v --durations=10 -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/full/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/full/pytest_gpu.log
# FETCH_SIZE pass first, so the bench line below carries roofline.traffic from it
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/full/pmc -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/full/pmc.log 2>&1 || { tail -20 gpurun_out/full/pmc.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/full/pmc/run_counter_collection.csv "${ROOF_KERNELS:-knn_chunk_lane_kernel,knn_lane_kernel}" 1024 2 1000000 1000000 gpurun_out/full/pmc.log > gpurun_out/full/traffic.log 2>&1 || { tail -5 gpurun_out/full/traffic.log; exit 1; }
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/full/bench.log 2>&1 || { tail -20 gpurun_out/full/bench.log; exit 1; }
tail -1 gpurun_out/full/bench.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/full/trace.log 2>&1 || { tail -20 gpurun_out/full/trace.log; exit 1; }
tail -1 gpurun_out/full/trace.log
cp profiles/knn_traffic.json gpurun_out/full/ 2>/dev/null || true
echo ok
