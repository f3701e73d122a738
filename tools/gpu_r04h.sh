# r04: C5's first-render cost (shard 1/8 cold, then shard 0/8 after a warmup render), and C4's
# shard 0/8 with the persistent Monte Carlo kernel on / off
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04h && mkdir -p $D
C5=(--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 "--extra=-dof 4 12.2282 0.025 -no_caustic" --no-cpu-baseline)
timeout -k 10 400 python3 -u bench.py "${C5[@]}" --shard 1/8 --steps 2 --warmup 0 > $D/c5_s1_cold.log 2>&1 || { tail -5 $D/c5_s1_cold.log; exit 1; }
tail -1 $D/c5_s1_cold.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C5 shard 1/8 cold steps", d["step_ms"])'
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline)
for p in 1024 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py "${C4[@]}" --shard 0/8 --steps 2 --warmup 1 > $D/c4_s0_$p.log 2>&1 || { tail -5 $D/c4_s0_$p.log; exit 1; }
  tail -1 $D/c4_s0_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C4 shard 0/8 persist=$p', d['value'], d['step_ms'], d['image_sha16'])"
done
echo ok
