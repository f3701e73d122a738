#!/bin/bash
# r05: row scatter fused with the launch-order keys (in-tree) against exp/base (FUSED_ROW_KEYS=0):
# parity suites, then interleaved C2 / C3 (tools/gpu_ab.sh), then one cold C2 frame trace each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05ae
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_configs.py tests/test_gpu_scenes.py tests/test_gpu_features.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_ab.sh 2 || exit 1
for f in gpurun_out/ab/c2.*.log; do grep '^{' $f | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', 'first', d['first_frame_ms'])"; done
exit $rc
