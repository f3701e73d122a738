#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c4ab
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --steps 1 --warmup 1 --shard 0/8 --no-cpu-baseline)
for v in base new; do
  L=""; [ $v = base ] && L=$GRAFT_REPO_ROOT/exp/base/libgi_amd.so
  GI_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py "${C4[@]}" > gpurun_out/c4ab/$v.log 2>&1 || { tail -5 gpurun_out/c4ab/$v.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/c4ab/$v.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', d['ms_per_step'], 'global', r['global']['avg_launch_ms'], 'caustic', r['caustic_kernel']['avg_launch_ms'], r['caustic_kernel'].get('fallback_avg_ms'))"
done
