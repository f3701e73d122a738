# r06 final tree: the whole GPU suite, the C2 bench line (with the CPU baseline) and the C5 shard
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/final_c
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 600 python3 -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-300
timeout -k 10 500 python3 -u bench.py --steps 2 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --no-cpu-baseline > $D/c5.log 2>&1 || { tail -5 $D/c5.log; exit 1; }
tail -1 $D/c5.log | cut -c1-300
