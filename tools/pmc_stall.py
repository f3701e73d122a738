"""Per-kernel wave-cycle split from one SQ PMC pass (tools/gpu_pmc_stall.sh): the fractions of
wave cycles parked on s_waitcnt (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY) and issuing
(SQ_ACTIVE_INST_ANY; MI355X_MICROARCH.md: the three are disjoint and sum to SQ_WAVE_CYCLES),
VALU-issuing, and instructions per wave. usage: pmc_stall.py run_counter_collection.csv"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "rocprim" in n:
        n = "rocprim::" + ("onesweep" if "onesweep" in r["Kernel_Name"] else "other")
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    calls[n].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
tot = sum(v.get("SQ_WAVE_CYCLES", 0) for _, v in rows)
print(f"{'kernel':58s} {'cyc%':>5s} {'wait':>5s} {'istall':>6s} {'active':>6s} {'valu':>5s} {'VALU/wave':>9s} {'SMEM/wave':>9s}")
for n, v in rows[:24]:
    wc = v.get("SQ_WAVE_CYCLES", 0)
    if wc <= 0:
        continue
    w = max(v.get("SQ_WAVES", 1), 1)
    print(f"{n[-58:]:58s} {100 * wc / tot:5.1f} {v.get('SQ_WAIT_ANY', 0) / wc:5.2f} "
          f"{v.get('SQ_WAIT_INST_ANY', 0) / wc:6.2f} {v.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.2f} "
          f"{v.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.2f} {v.get('SQ_INSTS_VALU', 0) / w:9.0f} "
          f"{v.get('SQ_INSTS_SMEM', 0) / w:9.0f}")
