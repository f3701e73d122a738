#!/usr/bin/env python3
"""Summary of the r06 glass-layer analysis -> stdout (profiles/r06_glass_fit.txt).

1. fig_14a-c per-pixel noise solved from the figures' pairwise differences, against the device's
   sample-count candidates (tools/glass_explore.py cand_* renders in GLASS_DIR, two seeds each).
2. fig_12's Fresnel change against the restatement's path classes (tools/glass_decompose.py
   OUT.npz files given as arguments: the shipped split, and the split at the primary hit only).

usage: python tools/glass_fit.py GLASS_DIR decompose.npz [decompose_primary_only.npz]
"""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mc_figs as mf  # noqa: E402
import oracle_lib  # noqa: E402


def noise_candidates(gdir):
    masks = mf.noise_masks(oracle_lib.intersect)
    fv = mf.figure_noise(masks)
    print("== fig_14 per-pixel noise variance (8-bit gray), figures solved from pair differences")
    for k in ("glass", "mirror"):
        print(f"  figure {k:6s} v8 {fv[k][8]:7.2f} v32 {fv[k][32]:7.2f} v128 {fv[k][128]:7.2f}")
    wall = np.zeros_like(masks["glass"])
    print("  candidates (device renders, v = var(seed1 - seed2) / 2):")
    print(f"  {'candidate':14s} {'glass':>7s} {'mirror':>7s}  paths/px")
    for f in sorted(glob.glob(os.path.join(gdir, "cand_*.npz"))):
        x = np.load(f)["imgs"].astype(float).mean(-1)
        name = os.path.basename(f)[:-4]
        aa = int(name.split("_a")[1][0])
        k = int(name.split("_k")[1])
        v = [float((x[0] - x[1])[masks[r]].var() / 2) for r in ("glass", "mirror")]
        print(f"  {name:14s} {v[0]:7.2f} {v[1]:7.2f}  {k * 4 ** aa}")
    del wall


def fresnel_fit(paths):
    from pngio import read_png  # noqa: F401
    for path in paths:
        d = np.load(path)
        mk = d["mask"]
        fa = mf.figure("fig_12a").astype(float).mean(-1)[::-1]
        fb = mf.figure("fig_12b").astype(float).mean(-1)[::-1]
        B = 8
        n = 512 // B
        bm = mk.reshape(n, B, n, B).all((1, 3))

        def blk(x):
            return x.reshape(n, B, n, B).mean((1, 3))[bm]

        def g(k):
            return d[k] if k in d else np.zeros((512, 512))
        fd = blk(fb - fa)
        D0 = blk(g("on_0") - g("off_-1"))
        C1 = blk(g("on_1") + g("on_17"))
        C4 = blk(g("on_4") + g("on_20"))
        ours = blk(g("on_-1") - g("off_-1"))
        X = np.stack([D0, C1, C4], 1)
        w, res, _r, _s = np.linalg.lstsq(X, fd, rcond=None)
        s = float((fd * ours).sum() / (ours * ours).sum())
        print(f"== fig_12b - fig_12a against {os.path.basename(path)} ({len(fd)} glass blocks)")
        print(f"  means: figure {fd.mean():.3f}, ours {ours.mean():.3f}; parts: transmitted loss "
              f"{D0.mean():.3f}, in-path reflections {C1.mean():.3f}, reflected fan {C4.mean():.3f}")
        print(f"  single scale {s:.3f} corr {np.corrcoef(fd, ours)[0, 1]:.4f} residual "
              f"{((fd - s * ours) ** 2).sum():.1f} of {(fd ** 2).sum():.1f}")
        print(f"  class weights (loss, in-path, fan) = {np.round(w, 3).tolist()} residual "
              f"{float(res[0]) if len(res) else float('nan'):.1f}")


if __name__ == "__main__":
    noise_candidates(sys.argv[1])
    fresnel_fit(sys.argv[2:])
