# r06f: the whole -m gpu suite after the knob / variant pruning, then a C2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06f
GI_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/r06f/parity_l2.jsonl timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r06f/pytest.log 2>&1 || { tail -40 gpurun_out/r06f/pytest.log; exit 1; }
tail -3 gpurun_out/r06f/pytest.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06f/bench.log 2>&1 || { tail -20 gpurun_out/r06f/bench.log; exit 1; }
tail -1 gpurun_out/r06f/bench.log | cut -c1-400
# the persistent Monte Carlo kernel for hard-light scenes too (GI_MC_PERSIST=1) vs the default
OUT=r06f_persist ROUNDS=2 CFGS="c2" VAR=GI_MC_PERSIST=1 bash tools/r06/ab.sh
