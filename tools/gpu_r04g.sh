# r04: C2 frame-time stability (fresh processes, persistent Monte Carlo kernel on / off, per-step
# times), then C5's shard balance
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04g && mkdir -p $D
for i in 1 2; do for p in 1024 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $D/c2_${p}_$i.log 2>&1 || { tail -5 $D/c2_${p}_$i.log; exit 1; }
  echo "C2 mc=$p run $i $(tail -1 $D/c2_${p}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_ms"], d["image_sha16"])')"
done; done
bash tools/gpu_balance.sh c5
