# FETCH_SIZE calibration passes for tools/fetch_calib (one PMC pass each) + the TCC counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/calib
mkdir -p $D
timeout -k 10 60 rocprofv3 -L > $D/counters.txt 2>&1 || true
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_EA_RD[A-Z0-9_]*\|TCC_REQ[A-Z0-9_]*\|TCC_READ[A-Z0-9_]*" $D/counters.txt | sort -u > $D/tcc_rd.txt || true
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/p1 -o run -- ./tools/fetch_calib > $D/p1.log 2>&1 || { tail -5 $D/p1.log; exit 1; }
for c in ${EXTRA_PMC:-}; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $D/p_$c -o run -- ./tools/fetch_calib > $D/p_$c.log 2>&1 || { tail -5 $D/p_$c.log; exit 1; }
done
cat $D/tcc_rd.txt | tr '\n' ' '; echo
python3 - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/calib/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(d)))
    agg = {}
    for r in rows:
        k = (r["Kernel_Name"][:40], r["Counter_Name"])
        agg[k] = agg.get(k, 0.0) + float(r["Counter_Value"])
    for k, v in sorted(agg.items()):
        print(os.path.basename(os.path.dirname(d)), k, v)
PY
