# r04: single-pass photon tracing (parity tests + C4 map build time vs the 2-pass build) and the
# C2 GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread -k "single_pass or photon_maps or emission_per_light or c2_ or c4_with or device_set or large_map_prop or batch_rerun" > gpurun_out/r04c/tests.log 2>&1 || { tail -30 gpurun_out/r04c/tests.log; exit 1; }
tail -3 gpurun_out/r04c/tests.log
for m in 1 0; do
  GI_PHOTON_2PASS=$m timeout -k 10 300 python3 -u tools/map_time.py stilllife.scn 2000000 10000000 2 > gpurun_out/r04c/map_$m.log 2>&1 || { tail -5 gpurun_out/r04c/map_$m.log; exit 1; }
  tail -1 gpurun_out/r04c/map_$m.log
  GI_PHOTON_2PASS=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c/prof_$m -o run -- python3 tools/map_time.py stilllife.scn 2000000 10000000 1 > gpurun_out/r04c/prof_$m.log 2>&1 || { tail -5 gpurun_out/r04c/prof_$m.log; exit 1; }
done
echo ok
