#!/bin/bash
# r05: phased packed d2 + Hilbert-curve launch order (in-tree) against exp/base (r05 tree):
# parity suites on the in-tree library, then the interleaved C2 / C3 A/B (tools/gpu_ab.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05n
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_variants.py tests/test_gpu_render.py tests/test_gpu_configs.py tests/test_gpu_scenes.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_ab.sh 2 || exit 1
grep -h '"global"' /dev/null; for f in gpurun_out/ab/c2.*.log; do grep '^{' $f | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', 'global', r['global']['avg_launch_ms'], 'frac', r['frac'], 'caustic', r['caustic_kernel']['avg_launch_ms'])"; done
exit $rc
