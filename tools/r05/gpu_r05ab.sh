#!/bin/bash
# r05: device allocations of a C2 bench (GI_ALLOC_LOG=1), run three times back to back (later ones
# starts right after the first exits), to see which allocation waits and the peak footprint.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05ab
mkdir -p $D
for r in 1 2 3; do
  GI_ALLOC_LOG=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/c2_$r.log 2>&1 || { tail -5 $D/c2_$r.log; exit 1; }
  grep '^{' $D/c2_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $r', d['ms_per_step'], 'first', d['first_frame_ms'])"
  grep "\[gi\] alloc" $D/c2_$r.log | awk '{s+=$3} END {print "allocated GB (sum of final sizes logged):", s}'
  grep "\[gi\] alloc" $D/c2_$r.log | sort -t: -k3 -n | tail -2
done
