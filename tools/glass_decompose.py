#!/usr/bin/env python3
"""Path-class decomposition of the glass sphere's pixels in jensen.scn, on
the oracle restatement (CPU; oracle_set_diag). For fig_12 / fig_14's configuration (512^2,
-no_indirect -no_caustic, -tt/-st N) every Monte Carlo contribution is rendered by class:

  fan 0 = TransmissiveIllumination's paths (raytracer.cpp:47-77),
  fan 1 = SpecularIllumination's Fresnel-reflected paths of the glass (raytracer.cpp:80-109 with
          R_coeff > 0, raytracer.cpp:204-219),
  event bits: +1 the path took a Fresnel reflection inside MonteCarlo_PathTrace
          (montecarlo.cpp:139-155 with R_coeff > 0), +2 a total internal reflection
          (TransmissiveBounce's fallback, graphics_utils.cpp:141-145),
  +16 when the contributing hit is the emissive light object.

For each class: its mean level over the glass sphere's interior pixels and its per-sample
variance A (per-pixel variance over seeds x N), with and without the Fresnel split, so that
the reference figures' anomalies (fig_12's Fresnel change 0.36 of ours; fig_14's glass noise
~2.4x ours) can be laid against the classes.

usage: python tools/glass_decompose.py OUT.json [N] [seeds] [aa] [extra flags...] [--no-mc-fresnel]
OUT.npz beside OUT.json keeps each class's seed-mean image (gray, 8-bit units, row 0 = bottom).
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402
import photon_figs as pf  # noqa: E402

SCN = os.path.join(ROOT, "tests", "scenes", "jensen.scn")
RES = 512
CLASSES = [0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18, 19, 20, 21, 22, 23]


def glass_mask():
    from scipy.ndimage import binary_erosion
    o, d = pf.camera_rays(SCN, RES, RES)
    hit, _t, _p, _n, m = oracle_lib.intersect(SCN, o, d)
    mat = np.where(hit > 0, m, -9).reshape(RES, RES)  # row 0 = bottom
    return binary_erosion(mat == 3, iterations=4)


def render_class(cls, args, win):
    L = oracle_lib.lib()
    L.oracle_set_diag.argtypes = [C.c_int] * 5
    L.oracle_run_tags.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p, C.c_int,
                                  C.c_void_p, C.c_void_p, C.c_int64]
    L.oracle_set_diag(cls, *win)
    n, argv = oracle_lib._argv(args)
    tags = (C.c_int * 1)(-100)
    f = np.zeros((RES, RES, 3), np.float32)
    rc = L.oracle_run_tags(n, argv, tags, 1, f.ctypes.data, None, RES * RES)
    L.oracle_set_diag(-1, 0, 0, 0, 0)
    assert rc == 0, rc
    return f.mean(-1) * 255.0  # gray, 8-bit units, row 0 = bottom


def main():
    out = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    seeds = list(range(1, 1 + (int(sys.argv[3]) if len(sys.argv) > 3 else 4)))
    aa = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    extra = [x for x in sys.argv[5:] if x != "--no-mc-fresnel"]
    # hypothesis test: the Fresnel split at the primary hit only, none inside the paths
    oracle_lib.lib().oracle_set_diag_flags(1 if "--no-mc-fresnel" in sys.argv[5:] else 0)
    mk = glass_mask()
    ys, xs = np.nonzero(mk)
    win = (int(xs.min()), int(ys.min()), int(xs.max()) + 1, int(ys.max()) + 1)
    res = {"N": N, "aa": aa, "seeds": seeds, "window": win, "pixels": int(mk.sum())}
    thr = str(os.cpu_count() or 8)
    allmaps = {}
    for fr in ("on", "off"):
        flags = ["-no_indirect", "-no_caustic", "-tt", str(N), "-st", str(N)] + extra
        if fr == "off":
            flags.append("-no_fresnel")
        t0 = time.time()
        per = {}
        tot = []
        maps = {}
        for cls in [-1] + CLASSES:
            imgs = []
            for s in seeds:
                args = [SCN, "/tmp/gd.png", "-resolution", str(RES), str(RES), "-aa", str(aa),
                        "-seed", str(s), "-threads", thr] + flags
                full = render_class(cls, args, win)
                maps[cls] = maps.get(cls, 0) + full / len(seeds)
                imgs.append(full[mk])
            imgs = np.stack(imgs)
            level = float(imgs.mean())
            A = float(imgs.var(0, ddof=1).mean() * N)
            if cls == -1:
                tot = imgs
                res[f"{fr}_total"] = {"level": level, "A": A}
            elif level != 0.0 or A != 0.0:
                # covariance with the rest of the pixel (what this class adds to the total's A)
                rest = tot - imgs
                cov = float(((imgs - imgs.mean(0)) * (rest - rest.mean(0))).sum(0).mean()
                            / (len(seeds) - 1) * N)
                per[str(cls)] = {"level": level, "A": A, "cov_with_rest": cov}
        res[f"{fr}_classes"] = per
        allmaps[fr] = {k: v.astype(np.float32) for k, v in maps.items()
                       if k == -1 or str(k) in per}
        print(fr, json.dumps(res[f"{fr}_total"]), f"{time.time() - t0:.0f} s", flush=True)
        for k, v in per.items():
            print(f"  class {k:>2}: level {v['level']:7.3f}  A {v['A']:8.2f}  cov {v['cov_with_rest']:8.2f}",
                  flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    np.savez_compressed(os.path.splitext(out)[0] + ".npz", mask=mk,
                        **{f"{fr}_{k}": v for fr, d in allmaps.items() for k, v in d.items()})


if __name__ == "__main__":
    main()
