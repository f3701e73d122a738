# r06a: C2 bench with the topology / image-check fields, then the glass exploration renders
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06a
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06a/bench.log 2>&1 || { tail -20 gpurun_out/r06a/bench.log; exit 1; }
tail -1 gpurun_out/r06a/bench.log | cut -c1-600
SEEDS=1,2,3 timeout -k 10 700 python -u tools/glass_explore.py gpurun_out/r06a/glass a0_ a1_ fw_ a2_on_t > gpurun_out/r06a/glass.log 2>&1 || { tail -20 gpurun_out/r06a/glass.log; exit 1; }
tail -3 gpurun_out/r06a/glass.log
