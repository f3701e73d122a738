# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over the k-NN micro.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
M="python3 tools/knn_micro.py --leaf 64 --kernels ${KNN_KERNELS:-0,1} --modes 0 --iters 1 --n 2000000"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/trace -o run -- $M > gpurun_out/pmc/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc/sq -o run -- $M > gpurun_out/pmc/sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- $M > gpurun_out/pmc/fetch.log 2>&1 || exit 1
echo done
