# r06m: (1) a third chunk pass for the global map (GI_CHUNK_LANE3=1024: the large-K chunk kernel
# over what the 480 pass left) on C5 / C4 shards and C2; (2) surface keys for the global list's
# launch order (GI_SURF_KEY=1) on C2 / C3 / C5, after their exactness test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06m
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py tests/test_gpu_knn_variants.py -k 'launch_order or LANE3' > gpurun_out/r06m/pytest.log 2>&1 || { tail -20 gpurun_out/r06m/pytest.log; exit 1; }
tail -2 gpurun_out/r06m/pytest.log
OUT=r06m_l3 ROUNDS=1 CFGS="c5 c4 c2" VAR=GI_CHUNK_LANE3=1024 bash tools/r06/ab.sh || exit 1
OUT=r06m_sk ROUNDS=1 CFGS="c2 c3 c5" VAR=GI_SURF_KEY=1 bash tools/r06/ab.sh
