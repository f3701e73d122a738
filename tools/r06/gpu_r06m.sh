# r06m: surface keys for the global list's launch order (GI_SURF_KEY=1) against the 3-D curve:
# exactness test, then interleaved A/B on C2 / C3 (2 rounds) and C4 / C5 shards (1 round)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06m
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py -k launch_order > gpurun_out/r06m/pytest.log 2>&1 || { tail -20 gpurun_out/r06m/pytest.log; exit 1; }
tail -2 gpurun_out/r06m/pytest.log
OUT=r06m ROUNDS=2 CFGS="c2 c3" VAR=GI_SURF_KEY=1 bash tools/r06/ab.sh || exit 1
OUT=r06m_big ROUNDS=1 CFGS="c5 c4" VAR=GI_SURF_KEY=1 bash tools/r06/ab.sh
