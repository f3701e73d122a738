# r06c: per-pixel sample-count candidates for fig_14 (tools/glass_explore.py cand_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06c
SEEDS=1,2 timeout -k 10 700 python -u tools/glass_explore.py gpurun_out/r06c/glass cand_ > gpurun_out/r06c/glass.log 2>&1 || { tail -20 gpurun_out/r06c/glass.log; exit 1; }
tail -3 gpurun_out/r06c/glass.log
