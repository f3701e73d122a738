#!/usr/bin/env python3
"""fp64 VALU work of the path kernels: per kernel, from PMC passes and a
kernel-trace stats file of the same workload:
  fp64 FLOP = 64 lanes x (2 FMA_F64 + ADD_F64 + MUL_F64) instructions (rocprofv3's own FLOP
              definition, counter_defs.yaml; TRANS_F64 not counted as FLOP),
  achieved  = fp64 FLOP / the kernel's total duration, against the fp64 vector peak
              (78.6 TFLOP/s: AMD's MI355X figure, half the FP32 vector rate of
              MI355X_MICROARCH.md),
  VALU busy = SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / (duration x clock x 1024 SIMDs),
  f64 share = fp64 VALU instructions / all VALU instructions.
usage: pmc_fp64.py PMC_DIR KERNEL_STATS_CSV [clock_GHz]"""
import collections
import csv
import glob
import json
import sys

PEAK_F64 = 78.6e12


def main():
    root, stats = sys.argv[1], sys.argv[2]
    ghz = float(sys.argv[3]) if len(sys.argv) > 3 else 2.4
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = {}
    for r in csv.DictReader(open(stats)):
        k = r["Name"].split("(")[0].replace("void ", "")
        dur[k] = dur.get(k, 0.0) + float(r["TotalDurationNs"]) * 1e-9
    out = []
    for k, v in agg.items():
        if k not in dur or not v.get("SQ_INSTS_VALU"):
            continue
        f64i = v["SQ_INSTS_VALU_FMA_F64"] + v["SQ_INSTS_VALU_ADD_F64"] + v["SQ_INSTS_VALU_MUL_F64"]
        flop = 64 * (2 * v["SQ_INSTS_VALU_FMA_F64"] + v["SQ_INSTS_VALU_ADD_F64"] +
                     v["SQ_INSTS_VALU_MUL_F64"])
        d = dur[k]
        row = {"kernel": k, "duration_s": round(d, 4),
               "fp64_tflops": round(flop / d / 1e12, 3),
               "fp64_frac_of_peak": round(flop / d / PEAK_F64, 4),
               "valu_busy": round(v.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (d * ghz * 1e9 * 1024), 4),
               "f64_share_of_valu": round((f64i + v["SQ_INSTS_VALU_TRANS_F64"]) / v["SQ_INSTS_VALU"], 4),
               "valu_insts_per_wave": round(v["SQ_INSTS_VALU"] / max(1.0, v.get("SQ_WAVES", 0)), 1)
               if v.get("SQ_WAVES") else None}
        out.append(row)
    out.sort(key=lambda r: -r["duration_s"])
    for r in out[:12]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
