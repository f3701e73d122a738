# r06g: cold C4 shard as the box's first GPU process, then the C2 bench after the leaf-size fix,
# then the persistent Monte Carlo kernel (1024 blocks) for hard lights vs the default on C2 / C4
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r06/gpu_cold.sh c4 r06g || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06g/bench.log 2>&1 || { tail -20 gpurun_out/r06g/bench.log; exit 1; }
tail -1 gpurun_out/r06g/bench.log | cut -c1-300
OUT=r06g_persist ROUNDS=2 CFGS="c2 c4" VAR=GI_MC_PERSIST=1024 bash tools/r06/ab.sh
