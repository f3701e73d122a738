#!/bin/bash
# r05: global-list launch-order cells (GI_KEY_BITS_G 10 vs 16) at the C4 / C5 shards, and 10 vs 12
# at C2 (400 M slots), caustic list at its 16-bit default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05q
mkdir -p $D
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=r.get('caustic_kernel') or {}; print('$2', d['value'], d['ms_per_step'], 'global', r['global']['avg_launch_ms'], 'g p2', r['global'].get('second_pass_query_frac'), 'caustic', c.get('avg_launch_ms'), d['image_sha16'])"; }
for b in 10 16; do
  GI_KEY_BITS_G=$b timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 1 --warmup 1 > $D/c4_$b.log 2>&1 || { tail -5 $D/c4_$b.log; exit 1; }
  line $D/c4_$b.log "c4 G$b"
done
for b in 10 16; do
  GI_KEY_BITS_G=$b timeout -k 10 600 python3 -u bench.py --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --steps 1 --warmup 1 --no-cpu-baseline > $D/c5_$b.log 2>&1 || { tail -5 $D/c5_$b.log; exit 1; }
  line $D/c5_$b.log "c5 G$b"
done
for b in 10 12 10 12; do
  GI_KEY_BITS_G=$b timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$b.log 2>&1 || { tail -5 $D/c2_$b.log; exit 1; }
  line $D/c2_$b.log "c2 G$b"
done
