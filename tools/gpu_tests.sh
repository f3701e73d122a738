set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 -E "gfx|Marketing" > gpurun_out/rocminfo.txt || true
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ]; then
  timeout -k 10 600 python bench.py --res 256 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
  echo "bench rc=$?"; tail -5 gpurun_out/bench_small.log
fi
