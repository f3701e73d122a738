#!/bin/bash
# The whole -m gpu suite with the per-comparison parity log (GI_PARITY_LOG); no -x, so every
# failing test is listed. usage: tools/gpu_suite.sh [pytest target]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/suite
rm -f gpurun_out/suite/parity.jsonl
GI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/suite/parity.jsonl timeout -k 10 1000 python -u -m pytest ${1:-tests} -v --durations=20 -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/suite/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/suite/pytest.log | tail -40
exit $rc
