# SQ counters of the renderer's kernels over a short bench (caustic map empty by default, so the
# global chunk k-NN dominates); two PMC passes, each its own run; summary via tools/pmc_summary.py
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmck
mkdir -p $D
B="python3 bench.py --res ${RES:-512} --steps 1 --warmup 0 --no-cpu-baseline --caustic-photons ${CPH:-0}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $D/p$i -o run -- $B > $D/p$i.log 2>&1 || { tail -5 $D/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $D
