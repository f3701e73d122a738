# r04: where C5's first render goes (per-batch log of a cold 1/64 shard), and C4 shard kernel
# stats with the persistent Monte Carlo kernel on / off
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04i && mkdir -p $D
C5=(--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 "--extra=-dof 4 12.2282 0.025 -no_caustic" --no-cpu-baseline)
GI_BATCH_LOG=1 timeout -k 10 400 python3 -u bench.py "${C5[@]}" --shard 1/64 --steps 2 --warmup 0 > $D/c5_s1of64.log 2>&1 || { tail -5 $D/c5_s1of64.log; exit 1; }
grep "batch\|step_ms" $D/c5_s1of64.log | head -60 | cut -c1-200
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline)
for p in 1024 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c4prof_$p -o run -- python3 bench.py "${C4[@]}" --shard 0/8 --steps 1 --warmup 1 > $D/c4prof_$p.log 2>&1 || { tail -5 $D/c4prof_$p.log; exit 1; }
done
echo ok
