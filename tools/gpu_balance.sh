#!/bin/bash
# Shard balance of the 8-GPU tile interleave measured on one MI355X (bench.py --balance):
# every shard s/8 rendered in turn. usage: tools/gpu_balance.sh c2|c4|c5 [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/balance
C=$1; shift
case $C in
  c2) A=(--steps 3); T=200 ;;
  c4) A=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000
         --steps 1); T=300 ;;
  c5) A=(--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1
         "--extra=-dof 4 12.2282 0.025 -no_caustic" --steps 1 --warmup 0); T=1000 ;;
esac
timeout -k 10 $T python3 -u bench.py "${A[@]}" --balance 8 "$@" > gpurun_out/balance/$C.log 2>&1 || { tail -5 gpurun_out/balance/$C.log; exit 1; }
grep '^{' gpurun_out/balance/$C.log | tail -1 > gpurun_out/balance/$C.json
tail -1 gpurun_out/balance/$C.json
