#!/bin/bash
# Where the waves of each kernel spend their cycles on a C2 (or BENCH_ARGS) frame: one SQ PMC
# pass (wave cycles parked on s_waitcnt, issue-stalled, issuing; VALU / SALU / SMEM instruction
# counts), summarised per kernel by tools/pmc_stall.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmcstall${TAG:-}
mkdir -p $D
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES --output-format csv -d $D/p1 -o run -- $B > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
python3 tools/pmc_stall.py $D/p1/run_counter_collection.csv | tee $D/summary.txt
