#!/usr/bin/env python3
"""Diagnostic: split a caustic-layer figure's oracle render by the material of
each photon's first specular / transmissive bounce (oracle_run_tags), so the figure can be
fitted as a per-material gain vector instead of one level ratio.

usage: python3 tools/caustic_decompose.py FIG [angle:]OUT.npz [seed ...]
(angle: / emit: split by the incidence cosine |N.I| at the query / by the emission
direction's cosine to the light normal, in five bins, instead of by material)
Writes OUT.npz: tags, per seed the float layers [ntags, H, W, 3] (row 0 = bottom) reduced to
float block means and the full-resolution layers (for the per-pixel quantisation model)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "global-illumination_amd"))

import oracle_lib  # noqa: E402
import photon_figs as pf  # noqa: E402

TAGS = [-100, 3, 4, 5, 6, -1]   # all, glass, mirror, gloss sphere, frosty box, default material
ANGLE_TAGS = [-100, 100, 101, 102, 103, 104]   # all, |N.I| in [0, .2), [.2, .4), ... [.8, 1]
EMIT_TAGS = [-100, 200, 201, 202, 203, 204]    # all, emission cosine in [0, .2), ... [.8, 1]
PATH_TAGS = [-100, 301, 302, 303, 304, 305, 306]   # all, path classes (oracle photon_trace)


def render_tags(args, w, h, tags):
    L = oracle_lib.lib()
    L.oracle_run_tags.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_void_p, C.c_int,
                                  C.c_void_p, C.c_void_p, C.c_int64]
    a = ["oracle"] + list(args)
    argv = (C.c_char_p * len(a))(*[x.encode() for x in a])
    t = np.array(tags, dtype=np.int32)
    f = np.zeros((len(tags), h, w, 3), dtype=np.float32)
    rc = L.oracle_run_tags(len(a), argv, t.ctypes.data, len(tags), f.ctypes.data, None, w * h)
    assert rc == 0, rc
    return f


def main():
    name, out = sys.argv[1], sys.argv[2]
    tags = TAGS
    if out.startswith("angle:"):
        tags, out = ANGLE_TAGS, out[6:]
    elif out.startswith("emit:"):
        tags, out = EMIT_TAGS, out[5:]
    elif out.startswith("path:"):
        tags, out = PATH_TAGS, out[5:]
    seeds = [int(s) for s in sys.argv[3:]] or [1]
    threads = len(os.sched_getaffinity(0))
    res = {"tags": np.array(tags)}
    for s in seeds:
        t0 = time.time()
        args, w, h = pf.render_args(name, s, threads=threads)
        f = render_tags(args, w, h, tags)
        res[f"seed{s}"] = f.astype(np.float16)
        print(f"seed {s}: {time.time() - t0:.0f} s", flush=True)
        np.savez_compressed(out, **res)


if __name__ == "__main__":
    main()
