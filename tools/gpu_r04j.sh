# r04: C5 cold render with buffer growth headroom (per-batch log of a 1/64 shard; shard 1/8
# cold and warm)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04j && mkdir -p $D
C5=(--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 "--extra=-dof 4 12.2282 0.025 -no_caustic" --no-cpu-baseline)
GI_BATCH_LOG=1 timeout -k 10 400 python3 -u bench.py "${C5[@]}" --shard 1/64 --steps 1 --warmup 0 > $D/c5_s1of64.log 2>&1 || { tail -5 $D/c5_s1of64.log; exit 1; }
grep "batch" $D/c5_s1of64.log | awk '{print $NF, $0}' | sort -rn | head -8 | cut -c1-180
tail -1 $D/c5_s1of64.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C5 1/64 cold", d["step_ms"])'
timeout -k 10 400 python3 -u bench.py "${C5[@]}" --shard 1/8 --steps 2 --warmup 0 > $D/c5_s1_cold.log 2>&1 || { tail -5 $D/c5_s1_cold.log; exit 1; }
tail -1 $D/c5_s1_cold.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("C5 shard 1/8 cold steps", d["step_ms"])'
echo ok
