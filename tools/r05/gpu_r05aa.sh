#!/bin/bash
# r05: bench's allocation probe before the first frame: three back-to-back C2 benches (the 2nd
# and 3rd start right after a ~100 GB process exits), first_frame_ms and alloc_probe_ms.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05aa
mkdir -p $D
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2_$r.log 2>&1 || { tail -5 $D/c2_$r.log; exit 1; }
  grep '^{' $D/c2_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $r', d['value'], d['ms_per_step'], 'first', d['first_frame_ms'], 'probe', d['alloc_probe_ms'])"
done
