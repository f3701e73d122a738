set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04a
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 > gpurun_out/r04a/bench.log 2>&1 && tail -1 gpurun_out/r04a/bench.log && bash tools/gpu_balance.sh c2 && bash tools/gpu_balance.sh c4
