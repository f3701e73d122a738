#!/bin/bash
# bench.py under several experiment libraries (exp/<name>/libgi_amd.so, tools/exp_build.sh),
# interleaved: VARIANTS="default csw5 ..." tools/gpu_variants.sh <bench args>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for r in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-default}; do
    if [ $v = default ]; then L=""; else L="GI_AMD_LIB=$GRAFT_REPO_ROOT/exp/$v/libgi_amd.so"; fi
    env $L timeout -k 10 400 python bench.py "$@" --no-cpu-baseline > gpurun_out/var/$v$r.log 2>&1 || { tail -5 gpurun_out/var/$v$r.log; exit 1; }
    echo "$v: $(grep '^{' gpurun_out/var/$v$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["roofline"]["global"]; c=d["roofline"]["caustic_kernel"]; print(d["ms_per_step"], "ms/frame; global", g["avg_launch_ms"], "caustic", c["avg_launch_ms"], "(fb", c["fallback_avg_ms"], ") sha", d["image_sha16"])')"
  done
done
