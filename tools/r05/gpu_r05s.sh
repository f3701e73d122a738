#!/bin/bash
# r05: global-list overflow handling re-tuned after the Hilbert order: C2 with the chunk kernel's
# sub-chunk floor (GI_CHUNK_MINSUB 32 default / 16 / 64) and without the 480-candidate second pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05s
mkdir -p $D
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['roofline']['global']; print('$2', d['value'], d['ms_per_step'], 'global', g['avg_launch_ms'], 'p2', g['second_pass_avg_ms'], g['second_pass_query_frac'], 'fb', g['fallback_avg_ms'], g['fallback_query_frac'], d['image_sha16'])"; }
for r in 1 2; do
for v in "def" "GI_CHUNK_MINSUB=16" "GI_CHUNK_MINSUB=64" "GI_CHUNK_LANE2=0"; do
  E=""; [ $v != def ] && E=$v
  env $E timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2.log 2>&1 || { tail -5 $D/c2.log; exit 1; }
  line $D/c2.log "$v $r"
done
done
