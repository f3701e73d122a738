#!/bin/bash
# Diagonal tile deal: multi-device / multi-rank / CLI GPU tests, then the C2 and C4 shard balance.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_cli.py tests/test_gpu_features.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/diag/pytest.log 2>&1 || { tail -30 gpurun_out/diag/pytest.log; exit 1; }
tail -2 gpurun_out/diag/pytest.log
bash tools/gpu_balance.sh c2 && mkdir -p gpurun_out/diag/b && cp gpurun_out/balance/c2.json gpurun_out/diag/b/ && bash tools/gpu_balance.sh c4 && cp gpurun_out/balance/c4.json gpurun_out/diag/b/
