# r06n: where the C2 frame time goes with surface keys (GI_SURF_KEY=1) against the 3-D curve:
# kernel-trace stats of one warm frame each, then two more interleaved A/B rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06n
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/base -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/base.log 2>&1 || { tail -20 $D/base.log; exit 1; }
tail -1 $D/base.log | cut -c1-200
GI_SURF_KEY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/sk -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/sk.log 2>&1 || { tail -20 $D/sk.log; exit 1; }
tail -1 $D/sk.log | cut -c1-200
OUT=r06n_ab ROUNDS=2 CFGS="c2" VAR=GI_SURF_KEY=1 bash tools/r06/ab.sh
