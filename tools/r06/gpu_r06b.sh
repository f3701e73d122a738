# r06b: glass / mirror shininess variants of jensen.scn (tools/glass_explore.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06b
SEEDS=1,2,3 timeout -k 10 700 python -u tools/glass_explore.py gpurun_out/r06b/glass gn mn a1_on_nodt a1_on_nods a1_off_nodt a1_off_nods > gpurun_out/r06b/glass.log 2>&1 || { tail -20 gpurun_out/r06b/glass.log; exit 1; }
tail -3 gpurun_out/r06b/glass.log
