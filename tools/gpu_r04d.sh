# r04: parity of the new paths (single-pass photon tracing, persistent Monte Carlo kernel, batch
# re-run, C2 tests), then A/B timings: C4 map build 2-pass vs 1-pass, C2 / C3 frame with the
# persistent Monte Carlo kernel on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04d && mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread -k "single_pass or photon_maps or emission_per_light or c2_ or batch_rerun or continuation_queue or full_gi or device_set" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -3 $D/tests.log
for m in 1 0; do
  GI_PHOTON_2PASS=$m timeout -k 10 300 python3 -u tools/map_time.py stilllife.scn 2000000 10000000 2 > $D/map_$m.log 2>&1 || { tail -5 $D/map_$m.log; exit 1; }
  tail -1 $D/map_$m.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_map -o run -- python3 tools/map_time.py stilllife.scn 2000000 10000000 1 > $D/prof_map.log 2>&1 || { tail -5 $D/prof_map.log; exit 1; }
for p in 1024 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_p$p.log 2>&1 || { tail -5 $D/c2_p$p.log; exit 1; }
  echo "C2 persist=$p $(tail -1 $D/c2_p$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 > $D/c3_p$p.log 2>&1 || { tail -5 $D/c3_p$p.log; exit 1; }
  echo "C3 persist=$p $(tail -1 $D/c3_p$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
done
echo ok
