#!/bin/bash
# r05: query-per-wave fallback's leaf-sweep height (SWEEP_H 6 in-tree vs 5 / 7 builds): C2 and
# the C4 shard caustic k-NN.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05ac
mkdir -p $D
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('$2', d['value'], d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'fb', c['fallback_avg_ms'], d['image_sha16'])"; }
for v in def sw5 sw7; do
  L=""; [ $v != def ] && L=$GRAFT_REPO_ROOT/exp/$v/libgi_amd.so
  GI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2.log 2>&1 || { tail -5 $D/c2.log; exit 1; }
  line $D/c2.log "c2 $v"
  GI_AMD_LIB=$L timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 1 --warmup 1 > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
  line $D/c4.log "c4 $v"
done
