# r06j: where C5's cold first frame goes (fresh box, first GPU process): allocation + batch log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06j
GI_LOG=3 timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --no-cpu-baseline > gpurun_out/r06j/c5.log 2>&1 || { tail -5 gpurun_out/r06j/c5.log; exit 1; }
grep -c "alloc" gpurun_out/r06j/c5.log; tail -1 gpurun_out/r06j/c5.log | cut -c1-200
