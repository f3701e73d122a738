#!/bin/bash
# C5 (teapot.scn 4096^2 aa 3, -dof 4 12.2282 0.025, 8 M global photons, -no_caustic: the default
# material is diffuse-only, so the caustic map would stay empty after ~10 futile emission rounds,
# SURVEY.md 8(d)) as ONE GPU's share of the 8-GPU frame: tile shard 0 of 8.
# A whole C5 frame on one GPU takes minutes (4.29 G pixel-samples); r02's attempt ran the whole
# frame under a time limit that killed it before the bench line was printed.
set -o pipefail
mkdir -p gpurun_out/c5
timeout -k 10 900 python -u bench.py --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 \
  --caustic-photons 1 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard ${SHARD:-0/8} \
  --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c5/c5_shard.log 2>&1
rc=$?
tail -c 3000 gpurun_out/c5/c5_shard.log
exit $rc
