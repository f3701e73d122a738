#!/usr/bin/env python3
"""Sum PMC counters per kernel over all counter_collection.csv files under a directory."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    if not v.get("SQ_WAVE_CYCLES"):
        continue
    print(k)
    wc = v["SQ_WAVE_CYCLES"]
    for c, x in sorted(v.items()):
        extra = f"  ({x / wc:.3f} of wave cycles)" if c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"   {c:36s} {x:14.4g}{extra}")
