"""CPU-baseline calibration: time the oracle
restatement on the survey's own C2 sample -- cornell.scn 64x64 aa 0, 1M global + 1M caustic
photons, 8 threads -- in the build container, against the reference binary's 72.62 s render on
the same sample and the same 8 cores (measured when the survey compiled it).

Test infrastructure: runs the oracle (tests/oracle_lib.py), never the product. Writes
profiles/<round>_cpu_calibration.json; bench.py's CPU_CALIBRATION quotes it.

usage: python tools/cpu_calibration.py [--round r05] [--repeats 2]
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import oracle_lib  # noqa: E402

REFERENCE_RENDER_S = 72.62     # 64^2 aa0 -threads 8, render
REFERENCE_MAP_S = 13.05        # same run, photon map (trace 12.08 + kd 0.97)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r05")
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    scene = os.path.join(ROOT, "tests", "scenes", "cornell.scn")
    args = [scene, "/tmp/calib.png", "-resolution", "64", "64", "-aa", "0", "-threads",
            str(a.threads), "-global", "1000000", "-caustic", "1000000", "-seed", "1"]
    runs = []
    for i in range(a.repeats):
        t0 = time.time()
        _rgb, st = oracle_lib.render(args, 64, 64)
        runs.append({"render_s": round(st["render_s"], 3), "trace_s": round(st["trace_s"], 3),
                     "kd_s": round(st["kd_s"], 3), "wall_s": round(time.time() - t0, 3),
                     "global_stored": int(st["global_stored"]),
                     "caustic_stored": int(st["caustic_stored"])})
        print(json.dumps(runs[-1]), flush=True)
    best = min(r["render_s"] for r in runs)
    out = {
        "sample": "cornell.scn 64x64 aa=0 -global 1000000 -caustic 1000000 -threads %d" % a.threads,
        "restatement_render_s": best,
        "restatement_map_s": min(r["trace_s"] + r["kd_s"] for r in runs),
        "reference_render_s": REFERENCE_RENDER_S,
        "reference_map_s": REFERENCE_MAP_S,
        "ratio": round(best / REFERENCE_RENDER_S, 3),
        "runs": runs,
        "cpu_model": cpu_model(),
        "cpus_visible": os.cpu_count(),
        "where": "build container (the reference binary's numbers are the survey's, same container)",
    }
    path = os.path.join(ROOT, "profiles", "%s_cpu_calibration.json" % a.round)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("restatement_render_s", "reference_render_s", "ratio")}))


if __name__ == "__main__":
    main()
