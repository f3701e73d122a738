#!/bin/bash
# Caustic k-NN A/B on a reduced C4 (stilllife 512^2 aa 2, 2M + 10M photons): the default build
# against GI_KNN_DBG=${AB_DBG:-1024} (the previous variant of the fallback), per-launch log lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
A="--scene stilllife.scn --res 512 --global-photons 2000000 --caustic-photons 10000000 --steps 2 --warmup 1 --no-cpu-baseline"
for v in new old; do
  if [ $v = old ]; then export GI_KNN_DBG=${AB_DBG:-1024}; else unset GI_KNN_DBG; fi
  GI_KNN_LOG=1 timeout -k 10 300 python bench.py $A > gpurun_out/ab/c4_$v.log 2>&1 || { tail -5 gpurun_out/ab/c4_$v.log; exit 1; }
  echo "== $v: $(grep '^{' gpurun_out/ab/c4_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["roofline"]["caustic_kernel"]; print(d["ms_per_step"], "ms/frame; caustic", c["avg_launch_ms"], "ms/launch, fallback", c["fallback_avg_ms"], "ms", c["fallback_query_frac"], "; sha", d["image_sha16"])')"
done
