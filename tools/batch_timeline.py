"""Per-batch kernel time split from a rocprofv3 kernel trace (batch = primary_kernel to the
next primary_kernel; times summed per kernel and stream). usage: batch_timeline.py trace.csv"""
import csv
import sys

KEYS = ["knn_chunk_big_kernel<512", "knn_chunk_big_kernel<1024", "knn_wave_kernel", "knn_chunk_lane",
        "knn_lane_kernel", "ind_cont", "ind_kernel", "mc_kernel", "slot0", "reduce_prim", "segments",
        "morton", "onesweep", "primary", "photon_kernel"]


def short(n):
    for k in KEYS:
        if k in n:
            return k.replace("knn_chunk_big_kernel", "big")
    return None


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prims = [i for i, r in enumerate(rows) if "primary_kernel" in r["Kernel_Name"]]
for bi, a in enumerate(prims):
    b = prims[bi + 1] if bi + 1 < len(prims) else len(rows)
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in rows[a:b])
    d = {}
    for r in rows[a:b]:
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        k += "/" + r["Stream_Id"]
        d[k] = d.get(k, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"batch {bi:2d} span {(t1 - t0) / 1e6:7.1f} ms: " +
          " ".join(f"{k}={v:.1f}" for k, v in d.items() if v >= 0.5))

# idle time: the part of each batch's span with no kernel running on any stream, and the largest
# gaps with the kernels on either side
for bi, a in enumerate(prims):
    b = prims[bi + 1] if bi + 1 < len(prims) else len(rows)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60])
                for r in rows[a:b])
    t0, end, idle, gaps = iv[0][0], iv[0][1], 0, []
    prev = iv[0][2]
    for s, e, n in iv[1:]:
        if s > end:
            idle += s - end
            gaps.append(((s - end) / 1e6, prev, n))
        if e > end:
            end, prev = e, n
    gaps.sort(reverse=True)
    print(f"batch {bi:2d} idle {idle / 1e6:6.2f} ms of {(end - t0) / 1e6:7.1f}; largest: " +
          "; ".join(f"{g:.2f} ms {p.split('(')[0][-28:]} -> {n.split('(')[0][-28:]}"
                    for g, p, n in gaps[:3]))
