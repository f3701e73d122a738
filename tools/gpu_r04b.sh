set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04b
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread -k c2_ > gpurun_out/r04b/c2tests.log 2>&1 || { tail -30 gpurun_out/r04b/c2tests.log; exit 1; }
tail -4 gpurun_out/r04b/c2tests.log
bash tools/gpu_balance.sh c5
