#!/bin/bash
# r05: finer launch-order cells (64-bit Hilbert keys) per list: exactness with both lists at 16
# bits, then C4 shard 0/8, C2 and C3 with the caustic list at 10 / 14 / 18 bits (GI_KEY_BITS_C).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05p
mkdir -p $D
GI_KEY_BITS_G=16 GI_KEY_BITS_C=16 timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_configs.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=r.get('caustic_kernel') or {}; print('$2', d['value'], d['ms_per_step'], 'global', r['global']['avg_launch_ms'], 'caustic', c.get('avg_launch_ms'), 'p2frac', c.get('second_pass_query_frac'), 'fbfrac', c.get('fallback_query_frac'), 'fb', c.get('fallback_avg_ms'), d['image_sha16'])"; }
for b in 10 14 18; do
  GI_KEY_BITS_C=$b timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 1 --warmup 1 > $D/c4_$b.log 2>&1 || { tail -5 $D/c4_$b.log; exit 1; }
  line $D/c4_$b.log "c4 C$b"
done
for b in 10 16; do
  GI_KEY_BITS_C=$b timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$b.log 2>&1 || { tail -5 $D/c2_$b.log; exit 1; }
  line $D/c2_$b.log "c2 C$b"
  GI_KEY_BITS_C=$b timeout -k 10 300 python3 bench.py --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3_$b.log 2>&1 || { tail -5 $D/c3_$b.log; exit 1; }
  line $D/c3_$b.log "c3 C$b"
done
exit $rc
