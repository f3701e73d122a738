#!/usr/bin/env python3
"""Photon-map build time (MapPhotons: tracing, power rescale, kd build, k-NN bounds) of one
configuration on the GPU, `reps` times over one context. Prints one JSON line per build.
usage: python3 tools/map_time.py SCENE GLOBAL CAUSTIC [reps]   (e.g. stilllife.scn 2000000 10000000)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import gi_amd  # noqa: E402


def main():
    scene, g, c = sys.argv[1], sys.argv[2], sys.argv[3]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    args = [os.path.join(ROOT, "tests", "scenes", scene), "/tmp/m.png", "-global", g,
            "-caustic", c, "-seed", "1"]
    p, sc, *_ = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(0, p)
    r.ReadScene(sc)
    for i in range(reps):
        t0 = time.perf_counter()
        st = r.MapPhotons()
        st["wall_s"] = time.perf_counter() - t0
        st["rep"] = i
        st["photon_2pass"] = os.environ.get("GI_PHOTON_2PASS", "0")
        print(json.dumps(st), flush=True)
    r.close()


if __name__ == "__main__":
    main()
