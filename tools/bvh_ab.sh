set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_features.py tests/test_gpu_render.py -m gpu -x -q --timeout 240 --timeout-method thread -k "mesh_bvh or intersections or full_gi_configs or stilllife or teapot" > gpurun_out/bvh_tests.log 2>&1 || { tail -30 gpurun_out/bvh_tests.log; exit 1; }
tail -3 gpurun_out/bvh_tests.log
for lib in ab/libgi_amd_nobvh.so global-illumination_amd/libgi_amd.so; do
  GI_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --scene teapot.scn --res 512 --aa 1 --global-photons 1000000 --extra "-no_caustic -dof 4 12.2282 0.025" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_teapot_$(basename $lib .so).json 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/bench_teapot_$(basename $lib .so).json
done
