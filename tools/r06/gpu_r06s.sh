# r06s: C4 shard 0/8 first frame on a fresh box, batch log (GI_LOG=2): where the first frame's
# extra time goes
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r06s
mkdir -p $D
GI_LOG=3 timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8 --no-cpu-baseline > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
tail -1 $D/c4.log | cut -c1-300
