#!/bin/bash
# Leaf slabs (KdView::slabs): exactness tests, then C4 shard 0/8 and C2 with GI_KD_SLABS=0 / 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/slabs
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_variants.py "tests/test_gpu_render.py::test_leaf_slabs_are_exact" -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/slabs/pytest.log 2>&1 || { tail -30 gpurun_out/slabs/pytest.log; exit 1; }
tail -3 gpurun_out/slabs/pytest.log
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --steps 1 --shard 0/8 --no-cpu-baseline)
for s in 0 1; do
  GI_KD_SLABS=$s timeout -k 10 300 python3 -u bench.py "${C4[@]}" > gpurun_out/slabs/c4_$s.log 2>&1 || { tail -5 gpurun_out/slabs/c4_$s.log; exit 1; }
  grep '^{' gpurun_out/slabs/c4_$s.log | tail -1 > gpurun_out/slabs/c4_$s.json
done
for s in 0 1; do
  GI_KD_SLABS=$s timeout -k 10 300 python3 -u bench.py --steps 5 --no-cpu-baseline > gpurun_out/slabs/c2_$s.log 2>&1 || { tail -5 gpurun_out/slabs/c2_$s.log; exit 1; }
  grep '^{' gpurun_out/slabs/c2_$s.log | tail -1 > gpurun_out/slabs/c2_$s.json
done
python3 - <<'PY'
import json
for c in ("c4", "c2"):
    for s in ("0", "1"):
        d = json.load(open(f"gpurun_out/slabs/{c}_{s}.json"))
        ck = d["roofline"]["caustic_kernel"]
        print(c, "slabs", s, "ms/step", d["ms_per_step"], "caustic ms/launch", ck["avg_launch_ms"],
              "2nd", ck.get("second_pass_avg_ms"), "fb", ck.get("fallback_avg_ms"),
              "visited/q", round(ck["visited_per_query"], 1), "sha", d.get("image_sha16"))
PY
