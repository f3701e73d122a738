set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in 0 1; do
  GI_SORT_QUERIES=$s timeout -k 10 600 python bench.py --res 256 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sort$s.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_sort$s.log
done
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; tail -3 gpurun_out/pytest_gpu.log
