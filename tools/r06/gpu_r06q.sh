# r06q: 64-bit surface keys for the caustic list (GI_SURF_KEY_C=1) against the 16-bit 3-D curve,
# with the global list's surface keys now the default: exactness, then C2 / C3 / C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06q
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py -k "launch_order" > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
OUT=r06q_ab ROUNDS=1 CFGS="c4 c2 c3" VAR=GI_SURF_KEY_C=1 bash tools/r06/ab.sh || exit 1
OUT=r06q_ab2 ROUNDS=1 CFGS="c2 c3" VAR=GI_SURF_KEY_C=1 bash tools/r06/ab.sh
