#!/bin/bash
# r05: scene walk without the per-element closest/scale division when scale == 1 (GI_SCALE_SKIP):
# parity suites on the new library, then the interleaved C2/C3 A/B against exp/base (=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05l
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_scenes.py tests/test_gpu_configs.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_ab.sh 2 || exit 1
exit $rc
