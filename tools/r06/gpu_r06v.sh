# r06v: the global map's last fallback as the query-per-wave kernel (GI_FB_WAVE=1) instead of
# the per-lane kernel: exactness (k-NN variants with the knob), C5 shard and C2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06v
mkdir -p $D
GI_FB_WAVE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_knn_variants.py -k "KERNEL7" > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
OUT=r06v_ab ROUNDS=1 CFGS="c5 c2" VAR=GI_FB_WAVE=1 bash tools/r06/ab.sh
