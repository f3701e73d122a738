set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof2
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --res 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 || exit 1
tail -1 gpurun_out/bench_small.log
for ls in ${GI_SWEEP_LEAF:-}; do
  GI_LEAF_SIZE=$ls timeout -k 10 600 python bench.py --res 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_leaf$ls.log 2>&1 || exit 1
  echo "leaf $ls: $(tail -1 gpurun_out/bench_leaf$ls.log | cut -c1-400)"
done
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --res 256 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof2/bench.log 2>&1 || exit 1
f=$(find gpurun_out/prof2 -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -c1-160 "$f" | head -14
