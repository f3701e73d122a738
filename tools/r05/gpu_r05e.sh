#!/bin/bash
# r05: the whole -m gpu suite (parity log), then C2's k-NN phase split (GI_KNN_DBG=16) and the
# VALU PMC pass of the k-NN kernels (tools/gpu_pmc_fp64.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_suite.sh
rc=$?
cp gpurun_out/suite/pytest.log gpurun_out/suite/pytest_r05e.log
[ $rc -le 1 ] || exit $rc
mkdir -p gpurun_out/r05e
GI_KNN_DBG=16 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r05e/c2_phase.log 2>&1 || { tail -5 gpurun_out/r05e/c2_phase.log; exit 1; }
grep "phase cycles" gpurun_out/r05e/c2_phase.log | tail -2
TAG=_r05e bash tools/gpu_pmc_fp64.sh
exit $rc
