#!/usr/bin/env python3
"""Score the device renders of tools/mc_figs_explore.py against the reference's Monte Carlo
transmissive / specular figures (fig_9b, fig_12, fig_14; gallery/tests specular / fourspheres):
for every (figure, candidate configuration) the photon-figure pin statistic (tests/photon_figs.py
pin: block z against the seeds, summed level) over ALL unsaturated blocks, and over the blocks
of the glass / mirror spheres alone (the layer under test), plus the per-pixel RMS against seed 1.

usage: python tools/mc_figs_fit.py DIR FIG_DIR [figure ...]
(FIG_DIR holds the figure PNGs; the committed copies are tests/golden/mc_figs/)
"""
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import photon_figs as pf  # noqa: E402
from pngio import read_png  # noqa: E402

# figure -> candidate-name prefix (tools/mc_figs_explore.py variants)
FIG_PREFIX = {
    "fig_9b-i": "j9_", "fig_9b-ii": "j9_", "fig_12a": "j_", "fig_12b": "j_",
    "fig_14a": "j_", "fig_14b": "j_", "fig_14c": "j_",
    "specular": "specular_", "fourspheres": "fourspheres_",
}


def blocks(img, B=16):
    n = img.shape[0] // B
    return img.astype(float).reshape(n, B, img.shape[1] // B, B, 3).mean((1, 3))


def main():
    d, figdir = sys.argv[1], sys.argv[2]
    figs = sys.argv[3:] or list(FIG_PREFIX)
    for fig in figs:
        fimg = read_png(os.path.join(figdir, fig + ".png"))[..., :3]
        fb = blocks(fimg)
        rows = []
        for path in sorted(glob.glob(os.path.join(d, FIG_PREFIX[fig] + "*.npz"))):
            z = np.load(path)
            sb = z["blocks"].astype(float)
            if sb.shape[1:] != fb.shape:
                continue
            first = z["first"].astype(float)
            mask = np.ones(fb.shape[:2], bool)
            r = pf.pin(fb, sb, mask)
            rms = float(np.sqrt(((first - fimg) ** 2).sum(-1).mean()))
            rows.append((r["median_abs_z"], os.path.basename(path)[:-4], r, rms))
        rows.sort(key=lambda t: t[0])
        print(f"== {fig}")
        for mz, name, r, rms in rows[:8]:
            print(f"  {name:24s} z_frac {r['z_frac']:.3f} med|z| {mz:6.2f} ratio {r['ratio']:.4f} "
                  f"(tol {r['ratio_tol']}) blocks {r['blocks']} rms1 {rms:6.2f} "
                  f"{'PASS' if r['ok'] else ''}")


if __name__ == "__main__":
    main()
