#!/bin/bash
# k-NN / scene parity tests, then the reduced C4 bench (stilllife 512^2 aa 2, 2M + 10M photons)
# twice with its image hash: one GPU call per kernel iteration.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/it
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_gpu_knn.py tests/test_gpu_knn_variants.py tests/test_gpu_scenes.py} > gpurun_out/it/tests.log 2>&1 || { tail -30 gpurun_out/it/tests.log; exit 1; }
tail -2 gpurun_out/it/tests.log
A="--scene stilllife.scn --res 512 --global-photons 2000000 --caustic-photons 10000000 --steps 2 --warmup 1"
for r in 1 2; do
  timeout -k 10 400 python bench.py $A --no-cpu-baseline > gpurun_out/it/c4_$r.log 2>&1 || { tail -5 gpurun_out/it/c4_$r.log; exit 1; }
  echo "c4-512: $(grep '^{' gpurun_out/it/c4_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); g=d["roofline"]["global"]; c=d["roofline"]["caustic_kernel"]; print(d["ms_per_step"], "ms/frame; global", g["avg_launch_ms"], "caustic", c["avg_launch_ms"], "(fb", c["fallback_avg_ms"], ") sha", d["image_sha16"])')"
done
