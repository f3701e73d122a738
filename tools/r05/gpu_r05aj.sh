#!/bin/bash
# r05: large-K chunk kernel occupancy target (BIG_WPE 3 in-tree vs 2 in exp/w2; LDS already caps
# the 512 instance at 9 waves per CU): C2 and the C4 shard, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05aj
mkdir -p $D
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('$2', d['value'], d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'p2', c['second_pass_avg_ms'], 'fb', c['fallback_avg_ms'], d['image_sha16'])"; }
for v in def w2; do
  L=""; [ $v = w2 ] && L=$GRAFT_REPO_ROOT/exp/w2/libgi_amd.so
  GI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2.log 2>&1 || { tail -5 $D/c2.log; exit 1; }
  line $D/c2.log "c2 $v"
  GI_AMD_LIB=$L timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 1 --warmup 1 > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
  line $D/c4.log "c4 $v"
done
