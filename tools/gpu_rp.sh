set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VARIANTS="default rpu8 rpu16" KPAT=reduce_prim,ind_kernel bash tools/gpu_variants_prof.sh --steps 1 --warmup 0 || exit 1
mkdir -p gpurun_out/rpmc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d gpurun_out/rpmc -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/rpmc/b.log 2>&1 || { tail -5 gpurun_out/rpmc/b.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/rpmc/**/*counter_collection.csv", recursive=True)[0]
agg = {}
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][-40:]
    d = agg.setdefault((k, r["Counter_Name"]), {})
    d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for (k, c), d in sorted(agg.items()):
    if any(x in k for x in ("reduce_prim", "ind_kernel", "slot0", "ind_cont")):
        print(f"{k:40s} {c:11s} n={len(d):3d} avg {sum(d.values())/len(d)/1e6:9.3f} (x1e6 KiB? raw units)")
PY
