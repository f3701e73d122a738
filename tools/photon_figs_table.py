#!/usr/bin/env python3
"""DESIGN.md 6.1's table: every photon-map figure pin from the committed oracle block statistics
(tests/golden/photon_figs/oracle_blocks.npz): blocks used, fraction with |z| < 3, median |z|,
figure / restatement level with its tolerance, the leave-one-out minimum of the |z| fraction.
usage: python3 tools/photon_figs_table.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import photon_figs as pf  # noqa: E402


def main():
    S = dict(np.load(pf.STATS))
    print("| figure | blocks | \\|z\\| < 3 | median \\|z\\| | figure / restatement (tol) "
          "| LOO min \\|z\\| < 3 | |")
    print("|---|---|---|---|---|---|---|")
    for name in list(pf.FIGS) + list(pf.EVIDENCE):
        if name + "/seeds" not in S:
            print(f"| {name} | GPU twin | | | | | |")
            continue
        seeds = S[name + "/seeds"].astype(float)
        r = pf.pin(S[name + "/figure"].astype(float), seeds, S[name + "/mask"])
        loo = min(x["z_frac"] for x in pf.leave_one_out(seeds, S[name + "/mask"]))
        print(f"| {name} | {r['blocks']} | {r['z_frac']:.3f} | {r['median_abs_z']:.2f} | "
              f"{r['ratio']:.3f} ({r['ratio_tol']:.2f}) | {loo:.3f} | "
              f"{'pass' if r['ok'] else 'miss'} |")


if __name__ == "__main__":
    main()
