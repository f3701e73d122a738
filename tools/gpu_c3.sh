# C3 (BASELINE.json configs[2]): jensen.scn 1024^2 aa=2, 4M caustic photons (global default
# 2176), one MI355X: the bench line and a kernel-trace profile of the same workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/c3
mkdir -p $D
A="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000"
timeout -k 10 600 python3 bench.py $A ${C3_BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline} > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
grep '^{' $D/bench.log | tail -1 > $D/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $A --steps 1 --warmup 1 --no-cpu-baseline > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
python3 tools/batch_timeline.py $D/trace/run_kernel_trace.csv | tail -12
cut -c1-1500 $D/bench.json
