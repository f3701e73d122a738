# Monte Carlo sub-path first-bounce kernel: parity (renders with glass vs the oracle, the
# continuation-queue exactness test) and C2 / C3 frames with and without it (image hashes equal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_features.py -m gpu -x -q --timeout 200 --timeout-method thread -k "full_gi or continuation or jensen or c5 or cache or fast_global or photon_viz" > gpurun_out/t_mcsub.log 2>&1 || { tail -20 gpurun_out/t_mcsub.log; exit 1; }
tail -1 gpurun_out/t_mcsub.log
STEPS=2 LIBS="default;exp/ms3/libgi_amd.so" bash tools/gpu_ab_lib.sh || exit 1
GI_MC_SUB=0 STEPS=2 bash tools/gpu_ab_lib.sh || exit 1
BENCH_ARGS="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000" LIBS="default;exp/ms3/libgi_amd.so" bash tools/gpu_ab_lib.sh || exit 1
GI_MC_SUB=0 BENCH_ARGS="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000" bash tools/gpu_ab_lib.sh
