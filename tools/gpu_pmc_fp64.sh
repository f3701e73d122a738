# fp64 VALU utilisation of the path kernels on a C2 (or BENCH_ARGS) frame: two PMC passes and a
# kernel-trace stats pass of the same command, summarised by tools/pmc_fp64.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmc64${TAG:-}
mkdir -p $D
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES" ; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $D/p$i -o run -- $B > $D/p$i.log 2>&1 || { tail -5 $D/p$i.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $B > $D/trace.log 2>&1 || { tail -5 $D/trace.log; exit 1; }
python3 tools/pmc_fp64.py $D $D/trace/run_kernel_stats.csv | tee $D/summary.jsonl
