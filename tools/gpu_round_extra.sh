set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIBS="default;exp/cw4/libgi_amd.so;exp/cw2/libgi_amd.so" STEPS=2 bash tools/gpu_ab_lib.sh || exit 1
LIBS="default;exp/cw4/libgi_amd.so" BENCH_ARGS="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000" bash tools/gpu_ab_lib.sh || exit 1
bash tools/gpu_c3.sh > /dev/null 2>&1 || exit 1
echo C3; tail -c 200 gpurun_out/c3/bench.json
bash tools/gpu_c5.sh > /dev/null 2>&1 || exit 1
echo C5; grep '^{' gpurun_out/c5/c5_shard.log | tail -1 | cut -c1-400
