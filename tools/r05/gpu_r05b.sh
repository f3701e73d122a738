#!/bin/bash
# r05: C4 shard 0/8 A/B of the path kernels' out-of-line scene walks (exp/ool{0,1,2}), then the
# cold first frame of C5 shard 1/8 and C2 with the batch and allocation logs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05b
mkdir -p $D
C4="--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8"
for l in exp/ool0/libgi_amd.so exp/ool1/libgi_amd.so exp/ool2/libgi_amd.so; do
  n=$(basename $(dirname $l))
  GI_AMD_LIB=$l timeout -k 10 300 python3 bench.py $C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/c4_$n.log 2>&1 || { tail -5 $D/c4_$n.log; exit 1; }
  grep '^{' $D/c4_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d['step_ms'], d['first_frame_ms'])"
done
C5="--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 --shard 1/8"
GI_BATCH_LOG=1 GI_ALLOC_LOG=1 timeout -k 10 400 python3 bench.py $C5 "--extra=-dof 4 12.2282 0.025 -no_caustic" --steps 1 --warmup 1 --no-cpu-baseline > $D/c5_cold.log 2>&1 || { tail -5 $D/c5_cold.log; exit 1; }
grep '^{' $D/c5_cold.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 shard1/8', d['ms_per_step'], 'first', d['first_frame_ms'])"
GI_BATCH_LOG=1 GI_ALLOC_LOG=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2_cold.log 2>&1 || { tail -5 $D/c2_cold.log; exit 1; }
grep '^{' $D/c2_cold.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], 'first', d['first_frame_ms'], d['image_sha16'])"
