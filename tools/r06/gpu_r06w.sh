# r06w: query-per-wave global fallback as the default: exactness (k-NN variants, render, configs,
# features), then without the 480 second pass (GI_CHUNK_LANE2=0) on C5 / C2 / C4, and C3 / C4
# with the new default against GI_FB_WAVE=0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06w
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_knn_variants.py tests/test_gpu_knn.py tests/test_gpu_render.py tests/test_gpu_configs.py > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
OUT=r06w_l2 ROUNDS=1 CFGS="c5 c2 c4" VAR=GI_CHUNK_LANE2=0 bash tools/r06/ab.sh || exit 1
OUT=r06w_fb ROUNDS=1 CFGS="c3 c4" VAR=GI_FB_WAVE=0 bash tools/r06/ab.sh
