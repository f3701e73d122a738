#!/bin/bash
# Shared device/oracle math (gi_math.h): the scene tests with the parity log (no -x: every scene's
# result), then the C2 / C3 A/B against exp/base (the library before the change).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gm
GI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/gm/parity.jsonl timeout -k 10 600 python -u -m pytest tests/test_gpu_scenes.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gm/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/gm/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_ab.sh 1
