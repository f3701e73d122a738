# C4 (stilllife.scn 2048^2 aa 2, 2M global + 10M caustic photons) on one MI355X: the whole frame
# (what the 8-GPU tile shard splits) and tile shard 0 of 8 (one GPU's share).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
A="--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline"
timeout -k 10 400 python3 bench.py $A --steps 1 --warmup 1 > gpurun_out/c4/full.log 2>&1 || { tail -5 gpurun_out/c4/full.log; exit 1; }
grep '^{' gpurun_out/c4/full.log | tail -1 > gpurun_out/c4/full.json
timeout -k 10 300 python3 bench.py $A --shard 0/8 --steps 1 --warmup 1 > gpurun_out/c4/shard.log 2>&1 || { tail -5 gpurun_out/c4/shard.log; exit 1; }
grep '^{' gpurun_out/c4/shard.log | tail -1 > gpurun_out/c4/shard0of8.json
for f in full shard0of8; do python3 -c "
import json; d=json.load(open('gpurun_out/c4/$f.json')); c=d['roofline']['caustic_kernel']
print('$f', d['value'], d['ms_per_step'], 'caustic ms/launch', c['avg_launch_ms'], 'fb frac', c['fallback_query_frac'], 'frac', d['roofline']['frac'])"; done
