#!/bin/bash
# GPU parity tests on the box: one pytest process, per-test timeout, log under gpurun_out/.
# usage: tools/gpu_tests.sh [pytest -k expression] [test files...]
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
shift || true
FILES=${@:-tests}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 1000 python -u -m pytest $FILES -m gpu -x -v --timeout 240 --timeout-method thread \
  "${KARG[@]}" > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
