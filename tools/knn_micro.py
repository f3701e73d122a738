#!/usr/bin/env python3
"""k-NN kernel micro-benchmark on realistic queries (GPU box diagnostics).

Photon maps: cornell.scn, 1M global + 1M caustic photons (bench.py's C2 maps).
Queries: surface points hit by rays from random points inside the box in random directions
(the distribution of Monte Carlo bounce vertices), Morton-ordered inside gi_knn_bench.
Prints one line per (leaf size, map, kernel, mode): ms per launch, ns per query, photons found
and photons visited per query.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4_000_000)
    ap.add_argument("--leaf", default="64")
    ap.add_argument("--kernels", default="0,1,2")
    ap.add_argument("--modes", default="0")
    ap.add_argument("--maps", default="0,1")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--capmul", default="1", help="GI_WAVE_CAP_MUL values")
    ap.add_argument("--slack", default="64", help="GI_SEL_SLACK values")
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    scene = os.path.join(ROOT, "tests", "scenes", "cornell.scn")
    combos = [(lf, cm, sl) for lf in a.leaf.split(",") for cm in a.capmul.split(",")
              for sl in a.slack.split(",")]
    for leaf, capmul, slack in combos:
        os.environ["GI_LEAF_SIZE"] = leaf
        os.environ["GI_WAVE_CAP_MUL"] = capmul
        os.environ["GI_SEL_SLACK"] = slack
        import gi_amd
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
        for mp in [int(x) for x in a.maps.split(",")]:
            for kern in [int(x) for x in a.kernels.split(",")]:
                for mode in [int(x) for x in a.modes.split(",")]:
                    ms, fq, vq = r.knn_bench(mp, pt, nr, mat, mode=mode, kernel=kern,
                                             iters=a.iters)
                    print(f"leaf={leaf} capmul={capmul} slack={slack} map={mp} kernel={kern} mode={mode} nq={len(pt)} "
                          f"ms={ms:.2f} ns/q={ms * 1e6 / len(pt):.2f} found={fq:.1f} "
                          f"visited={vq:.1f}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
