# r06 final tree: kernel-trace stats of the C2 bench (one warm frame)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/final_d
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
tail -1 $D/trace.log | cut -c1-200
