#!/usr/bin/env python3
"""Generate tests/golden/mc_figs/oracle_blocks.npz: the oracle restatement's 16 x 16 block means
of the Monte Carlo figure pins (tests/mc_figs.py FIGS and EVIDENCE) at mc_figs.SEEDS, the
figures' own block means, and the per-pixel agreement calibration (seed 1 against seed 2, and
the figure against seed 1). Test infrastructure: renders through tests/oracle_lib.py only.

usage: python3 tools/mc_figs_oracle.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import mc_figs as mf  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    threads = len(os.sched_getaffinity(0))
    out = {}
    for name in list(mf.FIGS) + list(mf.EVIDENCE):
        t0 = time.time()
        fig = mf.figure(name)
        out[name + "/figure"] = mf.blocks(fig).astype(np.float32)
        imgs = []
        for s in mf.SEEDS:
            args, w, h = mf.render_args(name, s, threads=threads)
            rgb, _st = oracle_lib.render(args, w, h)
            imgs.append(rgb[::-1].copy())
        out[name + "/seeds"] = np.stack([mf.blocks(i) for i in imgs]).astype(np.float32)
        # per-pixel agreement: [exact, <= 1 LSB] of seed 1 vs seed 2 and of the figure vs seed 1
        out[name + "/pix_seeds"] = np.array(mf.pixel_agreement(imgs[0], imgs[1]))
        out[name + "/pix_figure"] = np.array(mf.pixel_agreement(fig, imgs[0]))
        r = mf.pin(out[name + "/figure"].astype(float), out[name + "/seeds"].astype(float))
        print(f"{name}: {time.time() - t0:.0f} s  z_frac {r['z_frac']:.3f}  median|z| "
              f"{r['median_abs_z']:.2f}  ratio {r['ratio']:.5f}  pixels fig/seed1 "
              f"{out[name + '/pix_figure']}  seed1/seed2 {out[name + '/pix_seeds']}  "
              f"{'PASS' if r['ok'] else 'FAIL'}", flush=True)
    np.savez_compressed(mf.STATS, **out)


if __name__ == "__main__":
    main()
