#!/bin/bash
# r05: indirect-path kernel occupancy re-checked on the final tree (GI_IND_WAVES 4 default vs 3),
# C2 and C3 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05af
mkdir -p $D
for r in 1 2; do
  for v in 4 3; do
    GI_IND_WAVES=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2.log 2>&1 || { tail -5 $D/c2.log; exit 1; }
    grep '^{' $D/c2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 w$v $r', d['value'], d['ms_per_step'], d['image_sha16'])"
  done
done
for v in 4 3; do
  GI_IND_WAVES=$v timeout -k 10 300 python3 bench.py --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3.log 2>&1 || { tail -5 $D/c3.log; exit 1; }
  grep '^{' $D/c3.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 w$v', d['value'], d['ms_per_step'], d['image_sha16'])"
done
