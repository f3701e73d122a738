#!/bin/bash
# r05 first call: C3/C4/C5 exact-flag fixtures + full-size properties, the general-form guard,
# then the Monte Carlo figure exploration (tools/mc_figs_explore.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py "tests/test_gpu_knn_variants.py::test_general_form_miss_rerenders" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05a/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|assert" gpurun_out/r05a/pytest.log | tail -30
# 0 = passed, 1 = test failures: go on; anything else (timeout, crash) stops here
[ $rc -le 1 ] || exit $rc
SEEDS=6 timeout -k 10 900 python -u tools/mc_figs_explore.py gpurun_out/r05a/mcfig > gpurun_out/r05a/mcfig.log 2>&1 || { tail -5 gpurun_out/r05a/mcfig.log; exit 1; }
tail -3 gpurun_out/r05a/mcfig.log
# C3 with the indirect-queue clear moved before the fork: bench line + kernel stats (fills)
A=(--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline)
timeout -k 10 300 python3 bench.py "${A[@]}" --steps 3 --warmup 1 > gpurun_out/r05a/c3.log 2>&1 || { tail -5 gpurun_out/r05a/c3.log; exit 1; }
tail -1 gpurun_out/r05a/c3.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05a/c3trace -o run -- python3 bench.py "${A[@]}" --steps 1 --warmup 1 > gpurun_out/r05a/c3trace.log 2>&1 || { tail -5 gpurun_out/r05a/c3trace.log; exit 1; }
exit $rc
