#!/bin/bash
# Interleaved A/B of one bench.py configuration under two environments:
#   AB_A="VAR=x" AB_B="VAR=y" tools/gpu_ab_env.sh <bench args>
# runs A B A B (REPS pairs) and prints ms/frame, the k-NN launch times and the image hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abenv
for r in $(seq 1 ${REPS:-2}); do
  for v in A B; do
    E=$([ $v = A ] && echo "$AB_A" || echo "$AB_B")
    env $E timeout -k 10 400 python bench.py "$@" --no-cpu-baseline > gpurun_out/abenv/$v$r.log 2>&1 || { tail -5 gpurun_out/abenv/$v$r.log; exit 1; }
    echo "$v [$E]: $(grep '^{' gpurun_out/abenv/$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["roofline"]["global"]; c=d["roofline"]["caustic_kernel"]; print(d["ms_per_step"], "ms/frame; global", g["avg_launch_ms"], "caustic", c["avg_launch_ms"], "(fb", c["fallback_avg_ms"], ") sha", d["image_sha16"])')"
  done
done
