#!/bin/bash
# End-of-round C4 / C5 numbers: C4 shard balance (8 shards), C5 tile shard 1 of 8 (warm).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04r
bash tools/gpu_balance.sh c4 && cp gpurun_out/balance/c4.json gpurun_out/r04r/c4_shards.json || exit 1
timeout -k 10 400 python3 -u bench.py --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 "--extra=-dof 4 12.2282 0.025 -no_caustic" --steps 1 --warmup 1 --shard 1/8 --no-cpu-baseline > gpurun_out/r04r/c5.log 2>&1 || { tail -5 gpurun_out/r04r/c5.log; exit 1; }
grep '^{' gpurun_out/r04r/c5.log | tail -1 > gpurun_out/r04r/c5_shard1of8.json
python3 -c "
import json
d=json.load(open('gpurun_out/r04r/c5_shard1of8.json')); print('C5 shard 1/8', d['ms_per_step'], d['value'])
d=json.load(open('gpurun_out/r04r/c4_shards.json')); print('C4', d['max_ms'], d['mean_ms'], d['max_over_mean'], d['frame_Mpx_samples_per_s_at_N'])
"
