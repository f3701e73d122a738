"""Diagnostic: rays where the device's cylinder intersection differs from the oracle's
(cylinder.scn), saved for analysis on the CPU."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))
import gi_amd, oracle_lib
sc = os.path.join(ROOT, "tests", "scenes", "cylinder.scn")
r = gi_amd.Renderer(0)
r.ReadScene(sc)
rng = np.random.default_rng(0)
out = {}
for trial in range(4):
    n = 200000
    # emission-like rays from the two point lights toward the cylinder's neighbourhood
    light = np.array([[2, 2, 2], [-2, 2, 2]], float)[rng.integers(0, 2, n)]
    tgt = rng.normal(size=(n, 3)) * 0.8
    d = tgt - light
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    gh, gt, gp, gn, gm = r.Intersects(light, d)
    oh, ot, op, on, om = oracle_lib.intersect(sc, light, d)
    bad = (gh != oh) | ((gh == 1) & (oh == 1) & (np.abs(gt - ot) > 0))
    print("trial", trial, "hits", int(gh.sum()), "mismatch", int(bad.sum()), "hit-diff", int((gh != oh).sum()))
    for k, v in (("o", light), ("d", d), ("gh", gh), ("gt", gt), ("oh", oh), ("ot", ot), ("gn", gn), ("on", on)):
        out.setdefault(k, []).append(v[bad])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "cyl_mismatch.npz"), **{k: np.concatenate(v) for k, v in out.items()})
