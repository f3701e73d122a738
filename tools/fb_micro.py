#!/usr/bin/env python3
"""Caustic k-NN micro-benchmark on the queries that reach the query-per-wave fallback in a real
frame (GPU box). The queries come from tools/caustic_fb_dump.py (copied to exp/<tag>.npz, which
travels with the tree); the photon maps are rebuilt here with the same seed, so they are the
dumped ones. Queries are placed on the cornell floor's material with its normal (the fallback
queries' surface), radiance mode.

usage: tools/fb_micro.py [--npz exp/c2.npz] [--which fb] [--n 1000000] [--kernels 1,8]
Env knobs (GI_*) pass through; GI_KNN_DBG=16 prints the phase cycle counters.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npz", default=os.path.join(ROOT, "exp", "c2.npz"))
    ap.add_argument("--which", default="fb")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--kernels", default="1,8")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--scene", default="cornell.scn")
    ap.add_argument("--global-photons", type=int, default=1000000)
    ap.add_argument("--caustic-photons", type=int, default=1000000)
    a = ap.parse_args()
    import gi_amd
    z = np.load(a.npz)
    q = z[a.which][: a.n].astype(np.float64)
    nrm = np.zeros_like(q)
    nrm[:, 1] = 1.0
    mat = np.zeros(len(q), dtype=np.int32)
    scene = os.path.join(ROOT, "tests", "scenes", a.scene)
    args = [scene, "/tmp/x.png", "-global", str(a.global_photons), "-caustic", str(a.caustic_photons)]
    p, sc, _o, _w, _h, _aa, real = gi_amd.ParseArgs(args)
    r = gi_amd.Renderer(0, p)
    r.ReadScene(sc, real)
    r.MapPhotons()
    for kern in [int(x) for x in a.kernels.split(",")]:
        ms, fq, vq = r.knn_bench(1, q, nrm, mat, mode=0, kernel=kern, iters=a.iters)
        print(f"{a.which} n {len(q)} kernel {kern}: {ms:.2f} ms, {ms * 1e6 / len(q):.2f} ns/query, "
              f"found {fq:.1f} visited {vq:.1f}", flush=True)


if __name__ == "__main__":
    main()
