#!/bin/bash
# C3 (jensen 1024^2 aa 2, 4M caustic photons): bench line and kernel trace of the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c3final
A=(--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline)
timeout -k 10 300 python3 bench.py "${A[@]}" --steps 3 --warmup 1 > gpurun_out/c3final/bench.log 2>&1 || { tail -5 gpurun_out/c3final/bench.log; exit 1; }
tail -1 gpurun_out/c3final/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3final/trace -o run -- python3 bench.py "${A[@]}" --steps 1 --warmup 1 > gpurun_out/c3final/trace.log 2>&1 || { tail -5 gpurun_out/c3final/trace.log; exit 1; }
echo ok
