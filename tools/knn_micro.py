#!/usr/bin/env python3
"""k-NN kernel micro-benchmark on realistic queries (GPU box diagnostics).

Photon maps: cornell.scn, 1M global + 1M caustic photons (bench.py's C2 maps).
Queries: surface points hit by rays from random points inside the box in random directions
(the distribution of Monte Carlo bounce vertices), Morton-ordered inside gi_knn_bench.

Tuning knobs are environment variables read when a context is created (gi_host.cpp):
  --env GI_LEAF_SIZE=32,64 --env GI_LANE_CHUNK=4,8   sweeps their cartesian product.
Prints one line per (knob setting, map, kernel, mode): ms per launch, ns per query, photons
found and photons visited per query.
"""
import argparse
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4_000_000)
    ap.add_argument("--kernels", default="-1", help="-1 auto, 0 lane(old), 1 wave, 2 packet, 3 lane")
    ap.add_argument("--modes", default="0")
    ap.add_argument("--maps", default="0,1")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--env", action="append", default=[], help="NAME=v1,v2,...")
    a = ap.parse_args()
    names, values = [], []
    for e in a.env:
        k, v = e.split("=", 1)
        names.append(k)
        values.append(v.split(","))
    scene = os.path.join(ROOT, "tests", "scenes", "cornell.scn")
    import gi_amd
    for combo in (itertools.product(*values) if values else [()]):
        for k, v in zip(names, combo):
            os.environ[k] = v
        rng = np.random.default_rng(7)
        args = [scene, "/tmp/x.png", "-global", "1000000", "-caustic", "1000000"]
        p, sc, _o, w, h, aa, real = gi_amd.ParseArgs(args)
        r = gi_amd.Renderer(0, p)
        r.ReadScene(sc, real)
        r.MapPhotons()
        org = rng.random((a.n, 3)) * np.array([1.1, 1.09, 1.11])
        d = rng.normal(size=(a.n, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        hit, t, pt, nr, mat = r.Intersects(org, d)
        sel = hit != 0
        pt, nr, mat = pt[sel], nr[sel], mat[sel]
        tag = " ".join(f"{k}={v}" for k, v in zip(names, combo))
        for mp in [int(x) for x in a.maps.split(",")]:
            for kern in [int(x) for x in a.kernels.split(",")]:
                for mode in [int(x) for x in a.modes.split(",")]:
                    ms, fq, vq = r.knn_bench(mp, pt, nr, mat, mode=mode, kernel=kern,
                                             iters=a.iters)
                    print(f"{tag} map={mp} kernel={kern} mode={mode} nq={len(pt)} "
                          f"ms={ms:.2f} ns/q={ms * 1e6 / len(pt):.2f} found={fq:.1f} "
                          f"visited={vq:.1f}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
