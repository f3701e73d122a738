#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from a rocprofv3 `--pmc FETCH_SIZE` pass.

FETCH_SIZE is reported in KiB (rocprofv3 counter description). MI355X_MICROARCH.md (HBM
section): on gfx950 FETCH_SIZE reports 1/2 of the bytes actually read -> bytes = 2 * 1024 * KiB.
Writes profiles/knn_traffic.json, read by bench.py for roofline.traffic when the workload
matches.

usage: pmc_traffic.py <counter_collection.csv> <kernel-substring[,substring...]> <res> <aa>
                     <global> <caustic> [bench log of the PMC run]
The bench log (of the PMC run itself, --warmup 0, so that its k-NN stats cover every dispatch
the counters saw) gives the global map's query count: the traffic is kept as bytes per query,
and bench.py scales it by its own queries per launch (launch sizes follow the batch size).
Several substrings: the roofline "launch" is that sequence of kernels (e.g. the chunk kernel and
its per-lane fallback); their per-dispatch averages are summed.
"""
import csv
import json
import os
import sys


def main():
    path, knames = sys.argv[1], sys.argv[2].split(",")
    res, aa, glob, caus = (int(x) for x in sys.argv[3:7])
    nq = launches = None
    if len(sys.argv) > 7:
        for line in open(sys.argv[7]):
            if line.startswith("{"):
                g = json.loads(line)["roofline"]["global"]
                nq = g["queries_per_launch"] * g["launches"]
                launches = g["launches"]
    rows = list(csv.DictReader(open(path)))
    kib, ndisp, kib_all = 0.0, {}, 0.0
    for kname in knames:
        per = {}
        for r in rows:
            if kname not in r["Kernel_Name"] or r["Counter_Name"] != "FETCH_SIZE":
                continue
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        if not per:
            sys.exit(f"no FETCH_SIZE rows for {kname!r} in {path}")
        kib += sum(per.values()) / len(per)
        kib_all += sum(per.values())
        ndisp[kname] = len(per)
    out = {"kernel": " + ".join(knames), "dispatches": ndisp, "fetch_size_kib_per_launch": kib,
           "correction": "x2 (gfx950 FETCH_SIZE = 1/2 of bytes read, MI355X_MICROARCH.md) x1024",
           # one launch = the whole sequence (chunk passes + per-lane fallback) of one batch
           "bytes_per_launch": kib_all * 1024 * 2 / launches if launches else kib * 1024 * 2,
           "workload": {"res": res, "aa": aa, "global": glob, "caustic": caus},
           "queries": nq,
           "bytes_per_query": kib_all * 1024 * 2 / nq if nq else None,
           "source": os.path.relpath(path)}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "knn_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
