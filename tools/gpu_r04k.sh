# r04: persistent Monte Carlo kernel grid sweep (it shares the CUs with the main stream's path
# kernels): C2, C3 and C4's shard 0/8
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04k && mkdir -p $D
C3=(--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline)
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8)
for p in 128 256 512 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$p.log 2>&1 || { tail -5 $D/c2_$p.log; exit 1; }
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py "${C3[@]}" --steps 2 --warmup 1 > $D/c3_$p.log 2>&1 || { tail -5 $D/c3_$p.log; exit 1; }
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py "${C4[@]}" --steps 1 --warmup 1 > $D/c4_$p.log 2>&1 || { tail -5 $D/c4_$p.log; exit 1; }
  for c in c2 c3 c4; do echo "$c persist=$p $(tail -1 $D/${c}_$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["step_ms"], d["image_sha16"])')"; done
done
echo ok
