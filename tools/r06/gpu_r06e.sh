# r06e: k-NN exactness tests with the rank-placed bracket, then the interleaved A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_variants.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 || { tail -30 gpurun_out/r06e/pytest.log; exit 1; }
tail -2 gpurun_out/r06e/pytest.log
OUT=r06e ROUNDS=2 CFGS="c2 c3 c4" bash tools/r06/ab.sh
