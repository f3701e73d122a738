# r06d: the new figure pins and the multi-GPU bench tests on the device
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06d
GI_FIG_LOG=$GRAFT_REPO_ROOT/gpurun_out/r06d/figs.jsonl timeout -k 10 900 python -u -m pytest tests/test_gpu_mc_figs.py tests/test_gpu_multi.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06d/pytest.log 2>&1 || { tail -30 gpurun_out/r06d/pytest.log; exit 1; }
tail -3 gpurun_out/r06d/pytest.log
