# Kernel split of the caustic fallback microbenchmark (tools/fb_micro.py) under rocprofv3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fbprof
GI_KNN_LOG=1 GI_KNN_DBG=16 timeout -k 10 120 python tools/fb_micro.py --kernels 8 --iters 1 > gpurun_out/fbprof/log.txt 2>&1 || { tail -5 gpurun_out/fbprof/log.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/fbprof/log.txt | tail -6
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fbprof/trace -o run -- python3 tools/fb_micro.py --kernels 8 --iters 1 > gpurun_out/fbprof/trace.log 2>&1 || { tail -5 gpurun_out/fbprof/trace.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/fbprof/trace/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} {float(r["TotalDurationNs"])/1e6:9.2f} ms')
PY
