#!/bin/bash
# Interleaved A/B of the in-tree library against exp/base/libgi_amd.so (GI_AMD_LIB): C2 and C3
# benches, ROUNDS rounds of base/new, one JSON line per run into gpurun_out/ab/ab.jsonl.
# usage: tools/gpu_ab.sh [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.jsonl
C3=(--scene jensen.scn --global-photons 2176 --caustic-photons 4000000)
for r in $(seq 1 ${1:-2}); do
  for v in base new; do
    L=""; [ $v = base ] && L=$GRAFT_REPO_ROOT/exp/base/libgi_amd.so
    for c in c2 c3; do
      A=(--steps 3 --warmup 1 --no-cpu-baseline); [ $c = c3 ] && A+=("${C3[@]}")
      GI_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py "${A[@]}" > gpurun_out/ab/$c.$v.$r.log 2>&1 || { tail -5 gpurun_out/ab/$c.$v.$r.log; exit 1; }
      python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab/$c.$v.$r.log').read().strip().splitlines()[-1])
print(json.dumps({'cfg':'$c','v':'$v','round':$r,'ms':d['ms_per_step'],'step_ms':d.get('step_ms'),'sha':d.get('image_sha16')}))" >> gpurun_out/ab/ab.jsonl
    done
  done
done
cat gpurun_out/ab/ab.jsonl
