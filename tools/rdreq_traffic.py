#!/usr/bin/env python3
"""k-NN HBM read traffic from the TCC's EA read-request counters (cross-check of FETCH_SIZE x2).

FETCH_SIZE on gfx950 is (TCC_BUBBLE*128 + (TCC_EA0_RDREQ - TCC_BUBBLE - RDREQ_32B)*64 +
RDREQ_32B*32) / 1024 KiB (rocprofv3 -L), i.e. it prices every non-32-B request at 64 B, while
tools/fetch_calib shows the requests are 128 B for streaming reads and random 16-B gathers alike
(RDREQ_128B = one per 128-B line touched). This prices the requests by their own size class:
  bytes = 128 * RDREQ_128B + 64 * RDREQ_64B + 32 * RDREQ_32B
over the dispatches of the roofline kernels, per query of the global map (queries from the bench
log of the same run, as tools/pmc_traffic.py does).

usage: rdreq_traffic.py <counter_collection.csv> <kernel-substring[,...]> <bench log> [out.json]
"""
import csv
import json
import os
import sys

SIZES = {"TCC_EA0_RDREQ_128B_sum": 128, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_32B_sum": 32}


def main():
    path, knames, log = sys.argv[1], sys.argv[2].split(","), sys.argv[3]
    nq = None
    for line in open(log):
        if line.startswith("{"):
            g = json.loads(line)["roofline"]["global"]
            nq = g["queries_per_launch"] * g["launches"]
    tot = {c: 0.0 for c in list(SIZES) + ["TCC_EA0_RDREQ_sum"]}
    disp = {k: set() for k in knames}
    for r in csv.DictReader(open(path)):
        for k in knames:
            if k in r["Kernel_Name"] and r["Counter_Name"] in tot:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
                break
    if not nq or not any(disp.values()):
        sys.exit("no queries or no matching dispatches")
    b = sum(SIZES[c] * tot[c] for c in SIZES)
    out = {"kernel": " + ".join(knames), "dispatches": {k: len(v) for k, v in disp.items()},
           "counters": tot, "queries": nq, "bytes": b, "bytes_per_query": b / nq,
           "requests_per_query": tot["TCC_EA0_RDREQ_sum"] / nq,
           "source": os.path.relpath(path)}
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
