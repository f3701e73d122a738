#!/bin/bash
# Full GPU parity suite, then the C2 bench line and a short C3 line (timing A/B across changes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/check
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/check/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/check/pytest.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|E )" gpurun_out/check/pytest.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/check/c2.log 2>&1 || { tail -5 gpurun_out/check/c2.log; exit 1; }
grep '^{' gpurun_out/check/c2.log | cut -c1-420
timeout -k 10 600 python bench.py --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/check/c3.log 2>&1 || { tail -5 gpurun_out/check/c3.log; exit 1; }
grep '^{' gpurun_out/check/c3.log | cut -c1-420
