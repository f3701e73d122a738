# r04: per-batch times with the persistent Monte Carlo kernel on / off (GI_BATCH_LOG), C2 / C3 /
# C4 shard 0/8, to pick the batches it pays on
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04l && mkdir -p $D
C3=(--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline)
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8)
for p in 1024 0; do
  GI_BATCH_LOG=1 GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/c2_$p.log 2>&1 || { tail -5 $D/c2_$p.log; exit 1; }
  GI_BATCH_LOG=1 GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py "${C3[@]}" --steps 1 --warmup 1 > $D/c3_$p.log 2>&1 || { tail -5 $D/c3_$p.log; exit 1; }
  GI_BATCH_LOG=1 GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py "${C4[@]}" --steps 1 --warmup 1 > $D/c4_$p.log 2>&1 || { tail -5 $D/c4_$p.log; exit 1; }
done
echo ok
