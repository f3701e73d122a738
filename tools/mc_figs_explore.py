#!/usr/bin/env python3
"""Exploration for the Monte Carlo transmissive / specular figure pins:
render candidate configurations of the reference's fig_9b / fig_12 / fig_14 and
gallery/tests/specular.png / fourspheres.png on the device at several seeds and store the
8-bit renders' 16 x 16 block means, so that the captions' unstated settings (aa, sample counts,
Fresnel, distributed reflection) can be established on the CPU afterwards (tools/mc_figs_fit.py)
the way DESIGN.md 6.1 established the photon-map figures'.

The device renders equal the oracle restatement's bit for bit on the same seeds (the -m gpu
suite asserts that), so these blocks stand for the restatement's.

usage (GPU box): python tools/mc_figs_explore.py OUT_DIR [variant-prefix ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import gi_amd  # noqa: E402
from gpu_util import run_gpu  # noqa: E402

SCN = os.path.join(ROOT, "tests", "scenes")
B = 16
NOGI = ["-no_indirect", "-no_caustic"]


def variants():
    V = {}
    for aa in (0, 1, 2):
        for fr in ("on", "off"):
            f = [] if fr == "on" else ["-no_fresnel"]
            # fig_12: glass / mirror spheres in jensen.scn, Fresnel off (a) / on (b)
            V[f"j_aa{aa}_fr{fr}_mc"] = ("jensen.scn", 512, aa, NOGI + f)
            V[f"j_aa{aa}_fr{fr}_nodtds"] = ("jensen.scn", 512, aa, NOGI + f + ["-no_dt", "-no_ds"])
            # fig_14: Monte Carlo noise at 8 / 32 / 128 samples
            for n in (8, 32):
                V[f"j_aa{aa}_fr{fr}_t{n}"] = ("jensen.scn", 512, aa,
                                              NOGI + f + ["-tt", str(n), "-st", str(n)])
        # fig_9b: hard / soft shadows, black spheres
        V[f"j9_aa{aa}_hard"] = ("jensen.scn", 512, aa, NOGI + ["-no_transmissive", "-no_specular",
                                                               "-no_ss"])
        V[f"j9_aa{aa}_soft"] = ("jensen.scn", 512, aa, NOGI + ["-no_transmissive", "-no_specular"])
        # gallery/tests: specular.scn, fourspheres.scn (point / directional lights, no map)
        for sc in ("specular", "fourspheres"):
            V[f"{sc}_aa{aa}"] = (sc + ".scn", 512, aa, NOGI)
            V[f"{sc}_aa{aa}_nods"] = (sc + ".scn", 512, aa, NOGI + ["-no_ds"])
    V["j9_aa0_soft_lt512"] = ("jensen.scn", 512, 0, NOGI + ["-no_transmissive", "-no_specular",
                                                             "-lt", "512", "-ss", "512"])
    V["j9_aa1_soft_lt32"] = ("jensen.scn", 512, 1, NOGI + ["-no_transmissive", "-no_specular",
                                                            "-lt", "32", "-ss", "32"])
    V["j9_aa2_soft_lt8"] = ("jensen.scn", 512, 2, NOGI + ["-no_transmissive", "-no_specular",
                                                           "-lt", "8", "-ss", "8"])
    return V


def main():
    out = sys.argv[1]
    pref = sys.argv[2:]
    seeds = int(os.environ.get("SEEDS", "6"))
    os.makedirs(out, exist_ok=True)
    r = gi_amd.Renderer(0)
    V = variants()
    t00 = time.time()
    for name, (sc, res, aa, flags) in V.items():
        if pref and not any(name.startswith(p) for p in pref):
            continue
        t0 = time.time()
        blocks, first = [], None
        for s in range(1, seeds + 1):
            args = [os.path.join(SCN, sc), "/tmp/mf.png", "-resolution", str(res), str(res),
                    "-aa", str(aa), "-seed", str(s)] + flags
            rgb, _st, _ps = run_gpu(r, args)
            img = rgb[::-1]  # figure row order (top-down)
            n = res // B
            blocks.append(img.astype(float).reshape(n, B, n, B, 3).mean((1, 3)))
            if first is None:
                first = img.copy()
        np.savez_compressed(os.path.join(out, name + ".npz"), blocks=np.stack(blocks).astype(np.float32),
                            first=first, meta=json.dumps({"scene": sc, "res": res, "aa": aa,
                                                          "flags": flags}))
        print(f"{name}: {time.time() - t0:.1f} s (total {time.time() - t00:.0f} s)", flush=True)
    r.close()


if __name__ == "__main__":
    main()
