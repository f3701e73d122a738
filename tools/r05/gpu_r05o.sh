#!/bin/bash
# r05 configs after the Hilbert launch order: C3 frame, C4 tile shard 0/8, C5 tile shard 1/8.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${D:-gpurun_out/r05o}
mkdir -p $D
timeout -k 10 300 python3 bench.py --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3.log 2>&1 || { tail -5 $D/c3.log; exit 1; }
grep '^{' $D/c3.log | tail -1 > $D/c3.json
timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 2 --warmup 1 > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
grep '^{' $D/c4.log | tail -1 > $D/c4_shard0of8.json
timeout -k 10 600 python3 -u bench.py --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --steps 1 --warmup 1 --no-cpu-baseline > $D/c5.log 2>&1 || { tail -5 $D/c5.log; exit 1; }
grep '^{' $D/c5.log | tail -1 > $D/c5_shard1of8.json
for f in c3 c4_shard0of8 c5_shard1of8; do python3 -c "
import json; d=json.load(open('$D/$f.json')); r=d['roofline']; c=r.get('caustic_kernel') or {}
print('$f', d['value'], d['ms_per_step'], 'first', d.get('first_frame_ms'), 'global', r['global']['avg_launch_ms'], 'frac', r['frac'], 'caustic', c.get('avg_launch_ms'), 'fb', c.get('fallback_avg_ms'), d['image_sha16'])"; done
