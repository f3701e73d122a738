#!/bin/bash
# Kernel-trace of one bench.py configuration under several experiment libraries
# (exp/<name>/libgi_amd.so, tools/exp_build.sh; "default" = the product build), reporting the
# average time of the kernels matching KPAT (comma-separated substrings) and the image hash:
#   VARIANTS="default rp8" KPAT=reduce_prim tools/gpu_variants_prof.sh <bench args>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/vp
for r in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-default}; do
    if [ $v = default ]; then unset GI_AMD_LIB; else export GI_AMD_LIB=$GRAFT_REPO_ROOT/exp/$v/libgi_amd.so; fi
    D=gpurun_out/vp/$v$r
    timeout -k 10 ${TLIM:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py "$@" --no-cpu-baseline > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
    python3 - "$D" "$v" "${KPAT:-reduce_prim}" "$D.log" <<'PY'
import csv, glob, json, sys
d, v, pats, log = sys.argv[1], sys.argv[2], sys.argv[3].split(","), sys.argv[4]
rows = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0])))
line = [l for l in open(log) if l.startswith("{")][-1]
b = json.loads(line)
out = []
for p in pats:
    m = [r for r in rows if p in r["Name"]]
    n = sum(int(r["Calls"]) for r in m)
    t = sum(float(r["TotalDurationNs"]) for r in m)
    out.append(f"{p}: {t / max(n, 1) / 1e6:.3f} ms x {n}")
print(f"{v}: {b['ms_per_step']} ms/frame sha {b['image_sha16']} | " + " | ".join(out))
PY
  done
done
