# r04: the persistent Monte Carlo kernel with its dense, path-indexed sub-path queue: parity,
# C2 / C3 A/B and kernel stats; then the GPU twin of the photon-map figure pins
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04f && mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread -k "continuation_queue or full_gi or c2_config" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
C3="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline"
for p in 1024 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$p.log 2>&1 || { tail -5 $D/c2_$p.log; exit 1; }
  echo "C2 mc=$p $(tail -1 $D/c2_$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py $C3 --steps 2 --warmup 1 > $D/c3_$p.log 2>&1 || { tail -5 $D/c3_$p.log; exit 1; }
  echo "C3 mc=$p $(tail -1 $D/c3_$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
  GI_MC_PERSIST=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c3prof_$p -o run -- python3 bench.py $C3 --steps 1 --warmup 1 > $D/c3prof_$p.log 2>&1 || { tail -5 $D/c3prof_$p.log; exit 1; }
  GI_MC_PERSIST=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c2prof_$p -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/c2prof_$p.log 2>&1 || { tail -5 $D/c2prof_$p.log; exit 1; }
done
GI_FIG_LOG=$GRAFT_REPO_ROOT/$D/figs.jsonl timeout -k 10 900 python -u -m pytest tests/test_gpu_photon_figs.py -m gpu -v --timeout 600 --timeout-method thread > $D/figs.log 2>&1 || { tail -30 $D/figs.log; exit 1; }
tail -3 $D/figs.log
echo ok
