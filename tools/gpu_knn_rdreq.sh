# One PMC pass of the default bench (C2) with the TCC EA read-request size counters, priced by
# tools/rdreq_traffic.py: the k-NN kernels' own check of FETCH_SIZE x2 (see tools/fetch_calib.hip).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/rdreq
mkdir -p $D
timeout -k 10 -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $D/pmc -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
python3 tools/rdreq_traffic.py $D/pmc/run_counter_collection.csv knn_chunk_lane_kernel,knn_lane_kernel $D/pmc.log $D/knn_rdreq.json
