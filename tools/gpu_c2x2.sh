#!/bin/bash
# The default bench line (C2) twice, for a before/after comparison with a committed bench json.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c2x2
for r in 1 2; do
  timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/c2x2/b$r.log 2>&1 || { tail -5 gpurun_out/c2x2/b$r.log; exit 1; }
  grep '^{' gpurun_out/c2x2/b$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["roofline"]["global"]; c=d["roofline"]["caustic_kernel"]; print(d["value"], "Mpx/s", d["ms_per_step"], "ms/frame; global", g["avg_launch_ms"], "caustic", c["avg_launch_ms"], "sha", d["image_sha16"])'
done
